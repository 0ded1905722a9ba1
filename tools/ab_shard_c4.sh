#!/bin/bash
# Same-box A/B of build variants (multi-paxos_amd/lib_<v>/libmpx.so) against the default
# library on the C4 step and its 1-GPU shard projection, arms alternated, 3 rounds:
#   tools/ab_shard_c4.sh <tag> v1 [v2 ...]
set -o pipefail
tag=$1; shift
out=gpurun_out/ab_$tag
mkdir -p $out
rm -f $out/*.json
for rep in 1 2 3; do
  for v in default "$@"; do
    if [ $v = default ]; then unset MPX_LIB_VARIANT; else export MPX_LIB_VARIANT=$v; fi
    timeout -k 10 120 python bench.py --shard-only > $out/shard_${v}_$rep.json 2> $out/shard_${v}_$rep.err || { tail -5 $out/shard_${v}_$rep.err; exit 1; }
    timeout -k 10 200 python bench.py --no-cpu-baseline --c3-instances 0 --c5-instances 0 --c5c-instances 0 --shard-of 0 > $out/c4_${v}_$rep.json 2> $out/c4_${v}_$rep.err || { tail -5 $out/c4_${v}_$rep.err; exit 2; }
  done
done
unset MPX_LIB_VARIANT
python - $out <<'PY'
import json, glob, sys, collections
out = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(out + "/*.json")):
    name = f.split("/")[-1][:-5]
    kind, rest = name.split("_", 1)
    v = rest.rsplit("_", 1)[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])
    if kind == "shard":
        sp = d["scaling_projection"]
        res[v]["T_shard_us"].append(round(sp["T_shard_ms"] * 1e3, 2))
        res[v]["shard_phases"].append({k: round(x * 1e3, 1) for k, x in sp["phases_ms"].items()})
    else:
        res[v]["c4_ms"].append(round(d["ms_per_step"], 4))
        res[v]["c4_apply_ms"].append(round(d["roofline"]["kernel_ms"], 4))
summary = {v: {k: x for k, x in r.items()} for v, r in res.items()}
json.dump(summary, open(out + "/summary.json", "w"), indent=1)
for v, r in summary.items():
    print(v, "T_shard", r.get("T_shard_us"), "c4", r.get("c4_ms"))
PY

#!/bin/bash
# Same-box A/B on the C3 general-path leg (bench.py --c3-only), arms alternated, 3 rounds:
#   tools/ab_c3.sh <tag> v1 [v2 ...]       build variants (multi-paxos_amd/lib_<v>/libmpx.so)
#   tools/ab_c3.sh <tag> VAR=value [...]   environment switches on the default library
set -o pipefail
tag=$1; shift
out=gpurun_out/abc3_$tag
mkdir -p $out
rm -f $out/*.json
for rep in 1 2 3; do
  for v in default "$@"; do
    unset MPX_LIB_VARIANT
    envs=X=0
    case $v in default) ;; *=*) envs=$v ;; *) export MPX_LIB_VARIANT=$v ;; esac
    a=${v//=/_}
    env $envs timeout -k 10 300 python bench.py --c3-only > $out/c3_${a}_$rep.json 2> $out/c3_${a}_$rep.err || { tail -5 $out/c3_${a}_$rep.err; exit 1; }
  done
done
unset MPX_LIB_VARIANT
python - $out <<'PY'
import json, glob, sys, collections
out = sys.argv[1]
res = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(out + "/*.json")):
    v = f.split("/")[-1][:-5].split("_", 1)[1].rsplit("_", 1)[0]
    d = json.loads(open(f).read().strip().splitlines()[-1])["c3"]
    res[v]["ms_per_step"].append(round(d["ms_per_step"], 4))
    res[v]["general_ms"].append(round(d["phases_ms"]["general_apply"], 4))
    res[v]["fast_ms"].append(round(d["phases_ms"]["fast_apply"], 4))
    res[v]["digests"].append([d["verified"]["state_digest"], d["verified"]["chosen_digest"]])
json.dump(res, open(out + "/summary.json", "w"), indent=1)
for v, r in res.items():
    print(v, "step", r["ms_per_step"], "general", r["general_ms"], "fast", r["fast_ms"])
PY

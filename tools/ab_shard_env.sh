#!/bin/bash
# Same-library A/B of the 1-GPU shard projection (bench.py --shard-only) over environment
# switches, arms alternated, 3 rounds:  tools/ab_shard_env.sh <tag> VAR=value [VAR2=value ...]
# (arm "default" sets nothing; each other arm sets one VAR=value)
set -o pipefail
tag=$1; shift
out=gpurun_out/abenv_$tag
mkdir -p $out
rm -f $out/*.json
for rep in 1 2 3; do
  for kv in X=0 "$@"; do
    arm=${kv%%=*}_${kv#*=}
    env $kv timeout -k 10 120 python bench.py --shard-only > $out/${arm}_$rep.json 2> $out/${arm}_$rep.err || { tail -5 $out/${arm}_$rep.err; exit 1; }
  done
done
python - $out <<'PY'
import json, glob, sys, collections
out = sys.argv[1]
res = collections.defaultdict(list)
for f in sorted(glob.glob(out + "/*.json")):
    arm = f.split("/")[-1][:-5].rsplit("_", 1)[0]
    sp = json.loads(open(f).read().strip().splitlines()[-1])["scaling_projection"]
    res[arm].append({"T_shard_us": round(sp["T_shard_ms"] * 1e3, 2),
                     "phases_us": {k: round(x * 1e3, 1) for k, x in sp["phases_ms"].items()}})
json.dump(res, open(out + "/summary.json", "w"), indent=1)
for arm, r in res.items():
    print(arm, [x["T_shard_us"] for x in r], r[0]["phases_us"])
PY

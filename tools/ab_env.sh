# Bench A/B over an environment switch (same library), interleaved twice on one box:
#   tools/ab_env.sh VAR=value   (arm "on" sets it, arm "off" does not)
kv=$1
mkdir -p gpurun_out/ab_env
for rep in 1 2; do
  for arm in off on; do
    if [ $arm = on ]; then e="$kv"; else e="X=0"; fi
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_env/${arm}_$rep.json 2> gpurun_out/ab_env/${arm}_$rep.err || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_env/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"] * 1e3, 1), round(d["scaling_projection"]["T_shard_ms"] * 1e3, 1),
          round(d["c3"]["ms_per_step"], 4), round(d["c5"]["ms_per_step"], 4), d["verified"]["step_state_digest_vs_closed_form"])
PY

mkdir -p gpurun_out/ab_knob
for rep in 1 2; do
  for k in 0 1073741824; do
    MPX_KNOBS=$k timeout -k 10 200 python bench.py --no-cpu-baseline --c3-instances 0 --c5-instances 0 > gpurun_out/ab_knob/k${k}_$rep.json 2> gpurun_out/ab_knob/k${k}_$rep.err || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_knob/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["kernel_ms"] * 1e3, 1), round(d["scaling_projection"]["T_shard_ms"] * 1e3, 1), d.get("verified"))
PY

# Same-box A/B of the summary folded into k_store8 (default) vs its own k_reduce launch
# (MPX_KNOBS=1073741824): the C4 step and the 1-GPU shard projection, alternating arms
set -o pipefail
out=gpurun_out/ab_reduce
mkdir -p $out
rm -f $out/*.json
for rep in 1 2 3; do
  for k in 0 1073741824; do
    MPX_KNOBS=$k timeout -k 10 200 python bench.py --no-cpu-baseline --c3-instances 0 --c5-instances 0 > $out/c4_k${k}_$rep.json 2> $out/c4_k${k}_$rep.err || { tail -5 $out/c4_k${k}_$rep.err; exit 1; }
    MPX_KNOBS=$k timeout -k 10 120 python bench.py --shard-only > $out/shard_k${k}_$rep.json 2> $out/shard_k${k}_$rep.err || { tail -5 $out/shard_k${k}_$rep.err; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_reduce/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    if "ms_per_step" in d:
        print(f, "step_us", round(d["ms_per_step"] * 1e3, 1), "apply_us", round(d["roofline"]["kernel_ms"] * 1e3, 1), "verified", d.get("verified"))
    else:
        p = d["scaling_projection"]
        print(f, "T_shard_us", round(p["T_shard_ms"] * 1e3, 1), {k: round(v * 1e3, 1) for k, v in p["phases_ms"].items()}, "verified", p.get("verified"))
PY

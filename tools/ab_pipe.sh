# Same-box A/B of the pipelined C4 apply (LaunchGeom::pipe_stages: the plan of one bucket range
# beside the store of the previous one): stages x store workgroups per CU, the C4 step and the
# 1-GPU shard projection, arms alternated
set -o pipefail
out=gpurun_out/ab_pipe
mkdir -p $out
rm -f $out/*.json
arms="1:2 2:2 2:4 3:2 4:2 2:1"
for rep in 1 2; do
  for a in $arms; do
    st=${a%%:*}; pc=${a##*:}
    MPX_PIPE_STAGES=$st MPX_PIPE_STORE_PER_CU=$pc timeout -k 10 200 python bench.py --no-cpu-baseline --c3-instances 0 --c5-instances 0 > $out/c4_s${st}_w${pc}_$rep.json 2> $out/c4_s${st}_w${pc}_$rep.err || { tail -5 $out/c4_s${st}_w${pc}_$rep.err; exit 1; }
    MPX_PIPE_STAGES=$st MPX_PIPE_STORE_PER_CU=$pc timeout -k 10 120 python bench.py --shard-only > $out/shard_s${st}_w${pc}_$rep.json 2> $out/shard_s${st}_w${pc}_$rep.err || { tail -5 $out/shard_s${st}_w${pc}_$rep.err; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_pipe/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    if "ms_per_step" in d:
        v = d.get("verified") or {}
        print(f, "step_us", round(d["ms_per_step"] * 1e3, 1), "apply_us", round(d["roofline"]["kernel_ms"] * 1e3, 1), "ok", v.get("step_state_digest_vs_closed_form"), v.get("run_digests_vs_closed_form"))
    else:
        p = d["scaling_projection"]
        print(f, "T_shard_us", round(p["T_shard_ms"] * 1e3, 1), {k: round(x * 1e3, 1) for k, x in p["phases_ms"].items()}, "ok", p.get("verified"))
PY

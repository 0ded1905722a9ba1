# C4 (+ shard projection) A/B over build variants (multi-paxos_amd/lib_<v>/libmpx.so), one process per
# arm, interleaved twice on one box:  tools/ab_c4.sh v1 v2 ...
mkdir -p gpurun_out/ab_c4
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset MPX_LIB_VARIANT; else export MPX_LIB_VARIANT=$v; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --c3-instances 0 --c5-instances 0 --c5c-instances 0 > gpurun_out/ab_c4/${v}_$rep.json 2> gpurun_out/ab_c4/${v}_$rep.err || exit 1
  done
done
unset MPX_LIB_VARIANT
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_c4/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["ms_per_step"] * 1e3, 1), round(d["roofline"]["kernel_ms"] * 1e3, 1),
          round(d["scaling_projection"]["T_shard_ms"] * 1e3, 1))
PY

# A/B of a build variant (multi-paxos_amd/lib_<variant>/libmpx.so, same sources, other build
# knobs) against the default library: the shard projection and the full bench legs, one
# process per arm on the same box:  tools/ab_variant.sh <variant>
v=$1
mkdir -p gpurun_out/ab_$v
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py "${ARGS[@]}" > gpurun_out/ab_$v/$tag.json 2> gpurun_out/ab_$v/$tag.err || exit 1; }
ARGS=(--shard-only)
run shard_default X=0
run shard_$v MPX_LIB_VARIANT=$v
run shard_default2 X=0
run shard_${v}2 MPX_LIB_VARIANT=$v
ARGS=(--no-cpu-baseline)
run bench_default X=0
run bench_$v MPX_LIB_VARIANT=$v
python - "$v" <<'PY'
import json, glob, sys
for f in sorted(glob.glob("gpurun_out/ab_%s/*.json" % sys.argv[1])):
    d = json.load(open(f))
    sp = d.get("scaling_projection", {})
    line = {"T_shard_us": round(sp.get("T_shard_ms", 0) * 1e3, 1)}
    if "c3" in d:
        line.update(c4_ms=round(d["ms_per_step"], 4), c3_ms=round(d["c3"]["ms_per_step"], 4), c5_ms=round(d["c5"]["ms_per_step"], 4))
    print(f, line)
PY

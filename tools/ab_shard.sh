# A/B of the 1-GPU shard projection (bench.py --shard-only: rank 0's shard of C4 at world 8)
# over launch environment switches, one process per arm on the same box
mkdir -p gpurun_out/ab_shard
rm -f gpurun_out/ab_shard/*.json
run() { tag=$1; shift; env "$@" timeout -k 10 120 python bench.py --shard-only > gpurun_out/ab_shard/$tag.json 2> gpurun_out/ab_shard/$tag.err || exit 1; }
run default X=0
run events_every1000 MPX_EVENTS_EVERY=1000
run wgs1 MPX_STORE_WGS_PER_CU=1
run wgs4 MPX_STORE_WGS_PER_CU=4
run default2 X=0
for f in gpurun_out/ab_shard/*.json; do python -c "import json,sys; d=json.load(open('$f'))['scaling_projection']; print('$f', round(d['T_shard_ms']*1e3,1), {k: round(v*1e3,1) for k,v in d['phases_ms'].items()})"; done

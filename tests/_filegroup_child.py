"""Child process of test_dist_cpu.test_bench_filegroup_rendezvous (no torch import)."""
import os
import sys


def rank_main(rank, world, port, q):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_PORT"] = port
    import bench
    g = bench.FileGroup(rank, world)
    uid = bench.broadcast_bytes(g, b"uid-from-rank-0" if rank == 0 else None, rank)
    bench.barrier(g)
    mx = bench.allreduce_max(g, float(rank) * 1.5)
    g.close()
    q.put((rank, uid, mx))

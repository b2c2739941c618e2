"""Worker for tests/test_dist.py: one rank of the sharded MSM.

Each rank takes its contiguous shard [start, stop) of the point sequence
P_i = 2^(i+1) G and the matching slice of the seeded scalars, computes its
partial sum, then msm_blst_amd.dist exchanges the partial Jacobians
(all_gather) and folds them with an exact EC add.  Rank 0 prints the
compressed result.  MSM_DIST_COMPUTE selects who computes the partial:
  oracle  CPU restatement (oracle/liboracle.so) -- CPU test of the exchange path
  ches    the HIP CHES engine on cuda:0 (GPU test; ranks share one device)
  pip     the HIP plain Pippenger engine on cuda:0
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def main():
    import torch.distributed as dist

    group, n_total, seed = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    how = os.environ.get("MSM_DIST_COMPUTE", "oracle")
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()

    import msm_blst_amd as m
    from msm_blst_amd import dist as mdist

    start, stop = mdist.shard_range(n_total, world, rank)
    n = stop - start
    pts = m.fixed_points(group, n, start)
    sc_all = bytes(m.gen_scalars(n_total, seed))
    sc = sc_all[32 * start:32 * stop]

    def local():
        if how == "oracle":
            import ctypes

            import oracle_ffi as of
            S = (ctypes.c_uint8 * len(sc)).from_buffer_copy(sc)
            return bytes(of.msm(group, pts, S, n, 255, "pippenger"))
        if how == "ches":
            ctx = m.CHESContext(group, 0, n_exp=max(8, (n - 1).bit_length()))
            ctx.build_table(pts, n)
            r = ctx.mult(sc)
            ctx.close()
            return r
        ctx = m.MSMContext(group, 0, 12)
        ctx.set_points(pts, n)
        r = ctx.mult(sc, 255)
        ctx.close()
        return r

    res = mdist.sharded_msm(local, group)
    if rank == 0:
        print("RESULT", m.compress(group, res).hex(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

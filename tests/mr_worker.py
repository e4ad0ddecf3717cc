"""One rank of tests/test_gpu_multirank.py: a point shard solved through the
multi-rank exchange path of libba_hip with the host-staged transport
(ba_comm_init_host -> torch.distributed gloo), several ranks on one GPU."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    rank, world, port, out, lin, prec = (int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], Path(sys.argv[4]),
                                         sys.argv[5], sys.argv[6])
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bundleadjustment_amd import Options, Solver
    from test_gpu_multirank import scene, scene_bounds, solve_options
    from bundleadjustment_amd.problem import shard_points

    def allreduce(v, op):
        dist.all_reduce(torch.from_numpy(v), op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)

    name = sys.argv[7] if len(sys.argv) > 7 else "c2"
    p = scene(name)
    with Solver(0) as s:
        s.comm_init_host(allreduce, world, rank)
        s.set_problem(shard_points(p, world, rank, scene_bounds(p, world, name)))
        summ = s.solve(solve_options(lin, prec))
        cams, pts = s.params()
        log = s.iteration_log()
    np.savez(out / f"rank{rank}.npz", cams=cams, pts=pts, final=summ.final_cost,
             cost=np.array([r["cost"] for r in log]), cg=np.array([r["linear_solver_iterations"] for r in log]),
             ok=np.array([r["step_is_successful"] for r in log]))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

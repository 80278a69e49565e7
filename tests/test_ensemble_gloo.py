"""CPU, world_size 2 over gloo: the ensemble path (one independent analysis per rank, no inner-loop
communication, gather of the analyses to rank 0, max-over-ranks timing) that bench.py runs over RCCL."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, size, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(size), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "vae-var_amd"))
    sys.path.insert(0, os.path.join(root, "tests"))
    from test_host_logic import CpuPrims, objective
    from vaevar import ensemble
    from vaevar.lbfgs import LBFGS

    r, s, _ = ensemble.init("gloo")
    assert (r, s) == (rank, size)
    # an independent "analysis" per member: different problem (shifted objective) per rank
    z = torch.zeros(256)
    opt = LBFGS(CpuPrims(), z, history_size=10, max_iter=10, line_search_fn="strong_wolfe")

    def closure(zz, g):
        x = zz.clone().requires_grad_(True)
        f = objective(x - 0.1 * rank)
        f.backward()
        g.copy_(x.grad)
        return float(f)

    opt.step(closure)
    xs = ensemble.gather_analyses(z)
    tmax = ensemble.reduce_scalar(1.0 + rank, "max")
    iters = ensemble.reduce_scalar(opt.state["n_iter"], "sum")
    if rank == 0:
        q.put((torch.stack(xs).numpy(), tmax, iters))
    ensemble.barrier()
    torch.distributed.destroy_process_group()


def test_ensemble_gather_world2():
    size = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    xs, tmax, iters = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert xs.shape == (2, 256)
    assert tmax == 2.0 and iters >= 2
    # members solved different problems
    assert abs(xs[0] - xs[1]).max() > 1e-3


def test_member_assignment():
    from vaevar.ensemble import my_members

    assert my_members(8, 3, 8) == [3]
    assert my_members(10, 1, 4) == [1, 5, 9]
    assert sorted(sum((my_members(10, r, 4) for r in range(4)), [])) == list(range(10))

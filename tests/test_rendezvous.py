"""The torch-free host rendezvous of the one-process-per-GPU job (bench.py at
world > 1): unique-id broadcast, barrier and max-over-ranks, with 2 and 3
processes on CPU.  No torch is imported by the ranks."""
import multiprocessing as mp
import socket
import sys

import pytest

from conftest import REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, q):
    from dependence_free_rl_amd.rendezvous import Rendezvous
    r = Rendezvous(rank, world, addr="127.0.0.1", port=port, timeout=60)
    uid = r.broadcast(bytes(range(128)) if rank == 0 else None)
    r.barrier()
    m = r.allreduce_max(float(10 * rank + 1))
    r.barrier()
    r.close()
    q.put((rank, uid, m))


@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_star(world):
    port = _free_port()
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, uid, m in out:
        assert uid == bytes(range(128))
        assert m == float(10 * (world - 1) + 1)


def test_bench_world_path_imports_no_torch():
    """The modules bench.py's world > 1 path loads pull in no torch."""
    import subprocess
    code = ("import sys; import dependence_free_rl_amd.rendezvous; "
            "from dependence_free_rl_amd import Context, device_count; "
            "assert 'torch' not in sys.modules, 'torch imported'")
    subprocess.run([sys.executable, "-c", code], check=True, cwd=REPO)

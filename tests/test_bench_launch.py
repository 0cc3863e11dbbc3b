"""bench.py's N-rank launch without a GPU: `--gpus N`
with no WORLD_SIZE starts N rank processes itself (the parent never
initialises HIP), `--dry-run-ranks` runs each rank's env, rendezvous and
max-over-ranks time and stops before any HIP call; the same ranks under
torch.distributed.run; a device count below N fails fast; --gpus against a
different WORLD_SIZE is refused.  The ranks keep the reference's row-sum
semantics through the gradient SUM all-reduce (nn.h:94-98), replacing the
worker threads of apps/bin_packing/ppo_training.cc:48-62."""
import json
import os
import subprocess
import sys
import time

import pytest

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT",
                        "XH_RDZV_PORT")}
    env.update(kw)
    return env


def _check_dry(out, n):
    assert out.returncode == 0, (out.returncode, out.stderr[-2000:])
    lines = [l for l in out.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, out.stdout  # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["dry_run"] is True
    assert sorted(r["local_rank"] for r in d["ranks"]) == list(range(n))
    assert sorted(r["rank"] for r in d["ranks"]) == list(range(n))
    assert len({r["pid"] for r in d["ranks"]}) == n  # n processes
    envs = [json.loads(l.split("rank env: ", 1)[1])
            for l in out.stderr.splitlines() if "rank env: " in l]
    assert sorted(e["LOCAL_RANK"] for e in envs) == list(range(n))
    assert len({e["XH_RDZV_PORT"] for e in envs}) == 1  # one rendezvous
    # the max over ranks of the per-rank times (0.001 * (rank + 1))
    assert abs(d["max_rank_time_s"] - 0.001 * n) < 1e-12
    return d


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_launches_n_ranks(n):
    out = subprocess.run([sys.executable, BENCH, "--gpus", str(n),
                          "--dry-run-ranks"], capture_output=True, text=True,
                         env=_env(), timeout=120)
    _check_dry(out, n)


def test_dry_run_under_torch_distributed_run():
    """The driver's own form: torch.distributed.run sets WORLD_SIZE / RANK /
    LOCAL_RANK / MASTER_PORT; the rendezvous listens on MASTER_PORT + 1."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run",
                          "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port",
                          str(port), BENCH, "--gpus", "2", "--dry-run-ranks"],
                         capture_output=True, text=True, env=_env(),
                         timeout=180)
    _check_dry(out, 2)


def test_too_few_devices_fails_fast():
    """Here there is no GPU: --gpus 2 must stop in the parent with the
    device-count message instead of starting ranks that would hang in
    ncclCommInitRank."""
    t0 = time.monotonic()
    out = subprocess.run([sys.executable, BENCH, "--gpus", "2"],
                         capture_output=True, text=True, env=_env(),
                         timeout=60)
    if "needs 2 devices" not in out.stderr:
        pytest.skip("this host has >= 2 visible GPUs")
    assert out.returncode == 3 and out.stdout.strip() == ""
    assert time.monotonic() - t0 < 30


def test_gpus_must_match_world_size():
    out = subprocess.run([sys.executable, BENCH, "--gpus", "4"],
                         capture_output=True, text=True,
                         env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                         timeout=60)
    assert out.returncode == 2 and "disagrees with WORLD_SIZE" in out.stderr


def test_visible_device_count_reads_no_hip(monkeypatch):
    """The parent's device count reads sysfs and the visibility variables
    only (never the HIP runtime); a visibility list caps it."""
    sys.path.insert(0, REPO)
    import bench
    n = bench.visible_devices_no_hip()
    assert n >= 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert bench.visible_devices_no_hip() <= 1

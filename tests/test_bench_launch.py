"""bench.py's rank launch (`--gpus N` = N rank processes, the reference's `mpirun -np P`,
README:9), on the CPU: `--launch-check` runs the process group, barrier and max/sum
reductions of the bench line over gloo without any GPU leg."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                              "MASTER_PORT")}
    env["PJ_BENCH_BACKEND"] = "gloo"
    env["MASTER_ADDR"] = "127.0.0.1"
    return env


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_gpus_flag_starts_that_many_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                       timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["elapsed_max"] == 1.5  # max over ranks of 0.5 + rank
    assert d["units_sum"] == 30.0   # sum over ranks of 10 * (rank + 1)


def test_gpus_one_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--launch-check"], capture_output=True, text=True,
                       timeout=120, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_gpus_mismatching_the_launcher_fails():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", BENCH, "--gpus", "3", "--launch-check"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode != 0
    assert "--gpus 3 but the launcher started 2" in r.stderr


def test_partitioned_leg_guard_rejects_a_non_rccl_group():
    """at world > 1 the partitioned leg must run over an RCCL communicator
    whose own rank count (ncclCommCount) equals the world; the gloo rehearsal's host-buffer
    transport ("callbacks") is refused, and the refusal becomes the leg's error entry."""
    env = dict(_env(), PJ_BENCH_FORCE_PART="1")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"], capture_output=True, text=True,
                       timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    err = d["k28_partitioned"]["error"]
    assert "needs an RCCL communicator of 2 ranks" in err and "'callbacks' reporting 2" in err, err


def test_transport_guard_accepts_only_a_full_rccl_group():
    sys.path.insert(0, ROOT)
    import bench

    class C:
        def __init__(self, kind, count):
            self.kind, self._n = kind, count

        def transport_ranks(self):
            return self._n, 0

    assert bench.transport_guard(C("self", 1), 1) == {"transport": "self", "transport_ranks": 1, "transport_rank": 0}
    assert bench.transport_guard(C("rccl", 4), 4)["transport_ranks"] == 4
    for kind, n in (("rccl", 3), ("host", 4), ("callbacks", 4), ("self", 1)):
        try:
            bench.transport_guard(C(kind, n), 4)
        except RuntimeError as e:
            assert "needs an RCCL communicator of 4 ranks" in str(e)
        else:
            raise AssertionError((kind, n))

"""bench.py's own N-rank launcher (``python bench.py --gpus N`` without torch.distributed.run): the
decision taken before any GPU call, the environment each rank gets, and the parent's forwarding of
rank 0's result line and of the worst exit status.  CPU only: the ranks here are small Python
children standing in for the bench (the GPU run of the same path is ``CVAE_BENCH_SHARE_GPU=1
python bench.py --gpus 2`` in scripts/gpu_round.sh)."""
import io
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_plan_without_launcher():
    assert bench.launch_plan(None, {}, 0) == ("run", 1)
    assert bench.launch_plan(1, {}, 0) == ("run", 1)
    assert bench.launch_plan(8, {}, 8) == ("spawn", 8)
    assert bench.launch_plan(2, {"CVAE_BENCH_SHARE_GPU": "1"}, 1) == ("spawn", 2)


def test_plan_errors():
    what, msg = bench.launch_plan(8, {}, 1)
    assert what == "error" and "only 1 GPU" in msg
    what, msg = bench.launch_plan(0, {}, 8)
    assert what == "error"
    # a launcher's world that disagrees with --gpus would report the wrong n_gpus
    what, msg = bench.launch_plan(8, {"WORLD_SIZE": "1"}, 8)
    assert what == "error" and "WORLD_SIZE=1" in msg
    what, msg = bench.launch_plan(1, {"WORLD_SIZE": "x"}, 8)
    assert what == "error"


def test_plan_under_launcher():
    # the driver's form: torch.distributed.run --nproc-per-node N bench.py --gpus N
    assert bench.launch_plan(8, {"WORLD_SIZE": "8", "RANK": "3"}, 8) == ("run", 8)
    assert bench.launch_plan(None, {"WORLD_SIZE": "4"}, 8) == ("run", 4)
    # share mode under a launcher: the launcher's world, whatever the device count
    assert bench.launch_plan(4, {"WORLD_SIZE": "4", "CVAE_BENCH_SHARE_GPU": "1"}, 1) == ("run", 4)


def test_rank_envs():
    envs = bench.rank_envs(3, {"HSA_ENABLE_IPC_MODE_LEGACY": "0", "PATH": "/bin"}, 29999)
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    for e in envs:
        assert e["WORLD_SIZE"] == "3" and e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/bin"
    # every rank with the plan the bench takes under a launcher
    assert all(bench.launch_plan(3, e, 3) == ("run", 3) for e in envs)
    assert all("GPU_MAX_HW_QUEUES" not in e for e in envs)
    # ranks sharing one GPU: one hardware queue each (the GPU box exports HIP's default 4)
    shared = bench.rank_envs(2, {"CVAE_BENCH_SHARE_GPU": "1", "GPU_MAX_HW_QUEUES": "4"}, 29999)
    assert [e["GPU_MAX_HW_QUEUES"] for e in shared] == ["1", "1"]


CHILD = r"""
import json, os, sys
r = int(os.environ["RANK"])
print("banner on stdout", flush=True)            # native-library noise: not the result
print(json.dumps({"metric": "m", "value": 100 + r, "n_gpus": int(os.environ["WORLD_SIZE"])}), flush=True)
sys.exit(int(os.environ.get("FAIL_RANK_%d" % r, "0")))
"""


def _run(n, extra=None):
    env = dict(os.environ)
    env.update(extra or {})
    out = io.StringIO()
    rc = bench.run_ranks([sys.executable, "-c", CHILD], bench.rank_envs(n, env, 1), out, grace_s=5)
    return rc, out.getvalue()


def test_run_ranks_forwards_rank0_line():
    rc, out = _run(3)
    assert rc == 0
    lines = out.strip().splitlines()
    assert len(lines) == 1
    assert json.loads(lines[0]) == {"metric": "m", "value": 100, "n_gpus": 3}


def test_run_ranks_worst_status():
    rc, out = _run(3, {"FAIL_RANK_2": "3"})
    assert rc == 3
    assert json.loads(out)["value"] == 100  # rank 0's line still forwarded (the status says it failed)
    rc, _ = _run(2, {"FAIL_RANK_1": "5", "FAIL_RANK_0": "4"})
    assert rc == 4  # the first failing rank in rank order


def test_run_ranks_kills_stragglers():
    """A rank that fails while another waits (e.g. in a collective) does not hang the parent."""
    child = ("import os, sys, time\n"
             "r = int(os.environ['RANK'])\n"
             "sys.exit(7) if r == 1 else time.sleep(600)\n")
    out = io.StringIO()
    rc = bench.run_ranks([sys.executable, "-c", child], bench.rank_envs(2, dict(os.environ), 1), out, grace_s=1)
    assert rc == 7 and out.getvalue() == ""


def test_cli_mismatch_exits_before_gpu():
    """The real script: --gpus disagreeing with a launcher's WORLD_SIZE, or more GPUs than are
    visible, exits 2 with the reason before anything touches a GPU (none here)."""
    env = dict(os.environ)
    env.update({"WORLD_SIZE": "2", "RANK": "0"})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr and p.stdout == ""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "CVAE_BENCH_SHARE_GPU")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4096"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "GPU(s) are visible" in p.stderr and p.stdout == ""


def test_run_ranks_bounds_a_peer_left_behind_by_a_clean_exit():
    """rank 0 exits 0 while rank 1 hangs (e.g. in a collective rank 0 skipped) — the parent
    kills it after done_grace_s instead of polling forever."""
    child = ("import os, sys, time\n"
             "if os.environ['RANK'] == '1': time.sleep(60)\n"
             "sys.exit(0)\n")
    out = io.StringIO()
    t0 = time.monotonic()
    rc = bench.run_ranks([sys.executable, "-c", child], bench.rank_envs(2, dict(os.environ), 1), out, grace_s=1,
                         done_grace_s=1)
    assert time.monotonic() - t0 < 30
    assert rc != 0

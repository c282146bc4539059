"""bench.py's own N-rank launch (CPU): `python bench.py --gpus N` starts torch.distributed.run as
a child process when no launcher started it, decided before anything imports torch, and never
for one GPU or under an external launcher (WORLD_SIZE set)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _cmd(argv, env):
    return bench.launcher_command(bench.parse(argv), argv, env)


def test_one_gpu_never_spawns():
    assert _cmd([], {}) is None
    assert _cmd(["--gpus", "1", "--config", "C3"], {}) is None


def test_external_launcher_never_spawns():
    assert _cmd(["--gpus", "8"], {"WORLD_SIZE": "8", "RANK": "3"}) is None


def test_n_gpus_spawns_torchrun_with_the_same_arguments():
    argv = ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    cmd = _cmd(argv, {"MASTER_PORT": "29517"})
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd and "--master-port=29517" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1] == os.path.join(ROOT, "bench.py") and cmd[-len(argv):] == argv
    free = _cmd(["--gpus", "2"], {})
    port = int(free[[i for i, a in enumerate(free) if a.startswith("--master-port=")][0]].split("=")[1])
    assert 0 < port < 65536


def test_decision_imports_no_torch():
    # the parent decides and launches without importing torch (no device context to collide with)
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "c = bench.launcher_command(bench.parse(['--gpus', '2']), ['--gpus', '2'], {}); "
            "print(c is not None, 'torch' in sys.modules)" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["True", "False"]


def test_forwarder_passes_one_line_and_exit_status(capsys):
    ok = [sys.executable, "-c", "print('rank chatter'); print(%r)" % json.dumps({"metric": "m", "value": 1})]
    assert bench.run_launcher(ok) == 0
    out, err = capsys.readouterr()
    assert out.strip() == json.dumps({"metric": "m", "value": 1}) and "rank chatter" in err
    assert bench.run_launcher([sys.executable, "-c", "import sys; sys.exit(3)"]) == 3
    assert bench.run_launcher([sys.executable, "-c", "print('no line')"]) == 1


def test_device_shortfall_decision():
    assert bench.device_shortfall("nccl", 0, 1) is None
    assert bench.device_shortfall("nccl", 7, 8) is None
    assert "needs GPU 1" in bench.device_shortfall("nccl", 1, 1)
    assert bench.device_shortfall("nccl", 0, 0) is not None
    assert bench.device_shortfall("gloo", 5, 1) is None  # rehearsal ranks share the GPUs


def test_short_box_fails_fast_under_an_external_launcher():
    # one rank of an N-GPU job on a box with too few devices (here: none) exits non-zero with the
    # message, before any rendezvous
    env = dict(os.environ, WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29533",
               CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs GPU 1" in r.stderr and r.stdout.strip() == ""


def test_short_box_fails_fast_through_the_self_launch():
    # bench.py --gpus 2 starting its own ranks on a box with no visible device: every rank stops
    # before the rendezvous and the parent returns non-zero (no hang)
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0 and "needs GPU" in r.stderr, (r.returncode, r.stderr[-2000:])

"""CPU: the self-launch of the data-parallel ranks (vq3d/launch.py) -- `bench.py --gpus N` and
`python -m vq3d.train --gpus N` start their own N ranks under torch.distributed.run as a child
process, as the reference's Trainer(gpus=-1, accelerator='ddp') does (vqvae/train.py:25-27)."""
import json
import os
import subprocess
import sys
import textwrap

from conftest import PKG, ROOT

sys.path.insert(0, PKG)
from vq3d import launch  # noqa: E402
from vq3d import train as T  # noqa: E402


def _bench(*args, env=None, timeout=240):
    e = dict(os.environ if env is None else env)
    e.pop("WORLD_SIZE", None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=e)


def test_bench_self_launches_two_gloo_ranks():
    r = _bench("--gpus", "2", "--cpu-plumbing", "--steps", "3", "--warmup", "1")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # rank 0's line only; everything else goes to stderr
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["steps"] == 3 and line["warmup"] == 1 and line["allreduce_ok"]
    assert line["value"] > 0 and line["ms_per_step"] > 0


def test_bench_single_rank_does_not_launch():
    r = _bench("--gpus", "1", "--cpu-plumbing", "--steps", "2", "--warmup", "0")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["config"]["parallelism"] == "dp1"
    assert "torch.distributed.run" not in r.stderr


def test_failing_rank_propagates_exit_code(tmp_path):
    script = tmp_path / "fail_rank1.py"
    script.write_text(textwrap.dedent("""
        import os, sys
        print('{"rank": %s}' % os.environ["RANK"], flush=True)
        sys.exit(3 if os.environ["RANK"] == "1" else 0)
    """))
    rc = launch.run_ranks(2, str(script), [], json_only_stdout=True,
                          env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert rc != 0


def test_torchrun_command_shape():
    cmd = launch.torchrun_cmd(4, "bench.py", ["--gpus", "4"], port=29511)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-3:] == ["bench.py", "--gpus", "4"]
    assert launch.torchrun_cmd(2, "vq3d.train", [], module=True)[-2:] == ["-m", "vq3d.train"]


def test_resolve_gpus_forms(monkeypatch):
    monkeypatch.setattr(launch, "visible_gpus", lambda: 8)
    assert launch.resolve_gpus(None) == 0
    assert launch.resolve_gpus("1") == 1 and launch.resolve_gpus(4) == 4
    assert launch.resolve_gpus("-1") == 8 and launch.resolve_gpus(-1) == 8
    assert launch.resolve_gpus("0,1,3") == 3


def test_train_launch_decision(monkeypatch):
    calls = []
    monkeypatch.setattr(launch, "run_ranks", lambda n, entry, argv, module=False, env=None, **k:
                        calls.append((n, entry, module, env["PYTHONPATH"])) or 0)
    monkeypatch.setattr(launch, "visible_gpus", lambda: 8)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    argv = ["/data", "--gpus", "-1"]
    assert T.launch_ranks(T.parse_arguments(argv), argv) == 0  # the reference's default: every GPU
    assert calls[-1][:3] == (8, "vq3d.train", True)
    assert calls[-1][3].split(os.pathsep)[0] == os.path.realpath(PKG)
    assert T.launch_ranks(T.parse_arguments(["/data", "--gpus", "1"]), []) is None
    monkeypatch.setenv("WORLD_SIZE", "2")  # already a rank of a torchrun job
    assert T.launch_ranks(T.parse_arguments(argv), argv) is None


def test_train_cli_starts_ranks_end_to_end(tmp_path):
    """`python -m vq3d.train DATA --gpus 2` on this GPU-less host: both ranks start, import the
    package from this tree and stop at the GPU check; the launcher returns a failure code."""
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    env["PYTHONPATH"] = PKG
    r = subprocess.run([sys.executable, "-m", "vq3d.train", str(tmp_path), "--gpus", "2", "--max_steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode != 0
    assert r.stderr.count("a GPU is required") >= 2, r.stderr[-3000:]

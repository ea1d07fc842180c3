"""Self-launch of the data-parallel ranks: what the reference gets from PL's Trainer with
gpus=-1, accelerator='ddp' (vqvae/train.py:25-27) -- one command starts one process per GPU.

Standard library only, so an entry point can decide BEFORE importing torch or touching the
GPU: when more than one rank is wanted and the process is not already a rank (no WORLD_SIZE in
the environment), it starts `python -m torch.distributed.run --nproc-per-node N <entry> ...` as
a CHILD process (never an exec: a process that has initialised the GPU must not replace its
image), streams the child's output through and exits with the child's return code.  Under an
existing torchrun (WORLD_SIZE set) nothing happens and the caller runs as that rank.
"""
import json
import os
import signal
import socket
import subprocess
import sys


def is_rank_process():
    """True when this process already is one rank of a launched job (torchrun's env is set)."""
    return "WORLD_SIZE" in os.environ


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_gpus():
    """Number of GPUs a rank could use, counted in a throw-away child process so that this
    process never initialises the GPU itself (PL's gpus=-1 = every visible device)."""
    code = "import torch; print(torch.cuda.device_count() if torch.cuda.is_available() else 0)"
    try:
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        return int(out.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError, OSError):
        return 0


def resolve_gpus(spec):
    """PL's --gpus forms: None / 0 -> 0, an int N -> N, -1 or '-1' -> every visible GPU, a list
    '0,1,3' -> its length."""
    if spec is None:
        return 0
    s = str(spec).strip()
    if "," in s:
        return len([t for t in s.split(",") if t.strip()])
    n = int(s)
    return visible_gpus() if n < 0 else n


def torchrun_cmd(nproc, entry, args, module=False, port=None):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port or free_port())]
    cmd += (["-m", entry] if module else [entry]) + list(args)
    return cmd


def run_ranks(nproc, entry, args, module=False, json_only_stdout=False, env=None):
    """Run `entry` (a script path, or a module name with module=True) as `nproc` ranks under
    torch.distributed.run in a child process; return its exit code.

    json_only_stdout: forward only JSON-object lines to stdout (the bench contract: rank 0's one
    result line) and everything else to stderr."""
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL needs it)
    e.setdefault("MASTER_ADDR", "127.0.0.1")
    e["PYTHONUNBUFFERED"] = "1"
    # same process group as this launcher: a `timeout` around the launcher reaches the ranks too
    proc = subprocess.Popen(torchrun_cmd(nproc, entry, args, module=module), env=e, stdout=subprocess.PIPE,
                            text=True, bufsize=1)
    old = signal.signal(signal.SIGTERM, _raise_exit)
    try:
        for line in proc.stdout:
            if json_only_stdout and not _is_json_object(line):
                sys.stderr.write(line)
                sys.stderr.flush()
            else:
                sys.stdout.write(line)
                sys.stdout.flush()
        return proc.wait()
    except BaseException:
        # interrupted (Ctrl-C, SIGTERM): torchrun forwards the signal to its ranks and reaps them
        if proc.poll() is None:
            proc.terminate()
            try:
                proc.wait(timeout=60)
            except subprocess.TimeoutExpired:
                proc.kill()
        raise
    finally:
        signal.signal(signal.SIGTERM, old)


def _raise_exit(signum, frame):
    raise SystemExit(128 + signum)


def _is_json_object(line):
    s = line.strip()
    if not (s.startswith("{") and s.endswith("}")):
        return False
    try:
        return isinstance(json.loads(s), dict)
    except ValueError:
        return False

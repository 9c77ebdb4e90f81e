"""One process per GPU, started by the entry point itself (bench.py, main_imagenet.py).

The reference's data-parallel script spawns its own ranks: `ngpus_per_node =
torch.cuda.device_count(); mp.spawn(main_worker, nprocs=ngpus_per_node, ...)`
(Brecq/main_imagenet_dist.py:268-271).  Here `--gpus N` with N > 1 and no WORLD_SIZE in the
environment (no external torch.distributed.run) starts N fresh interpreters of the same
script, each with the environment torch.distributed.run would give it (RANK, LOCAL_RANK,
WORLD_SIZE, MASTER_ADDR=127.0.0.1, a free MASTER_PORT), and returns the first failing
rank's exit code (else 0).

This module imports nothing but the standard library, and the entry points call
`maybe_spawn` before they import torch: the parent never maps the HIP runtime, let alone
initialises a device, so no child is forked or exec'd from a process that touched the GPU.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

LAUNCHER_ENV = "SSQ_LAUNCHER"
# test hook: every spawned rank prints its rendezvous environment and exits before torch is
# imported; the parent prints what it had mapped when it spawned (tests/test_host.py)
DRYRUN_ENV = "SSQ_LAUNCH_DRYRUN"


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def hip_runtime_mapped():
    """True when this process has the HIP runtime (libamdhip64) mapped."""
    try:
        with open("/proc/self/maps") as f:
            return any("libamdhip64" in line for line in f)
    except OSError:
        return False


def parent_state():
    """What the spawning process holds: it must be nothing GPU-side."""
    torch = sys.modules.get("torch")
    cuda_init = bool(torch is not None and torch.cuda.is_initialized())
    return {"torch_imported": torch is not None, "cuda_initialized": cuda_init,
            "hip_runtime_mapped": hip_runtime_mapped(),
            "libssq_loaded": "shiftedscalequantization_amd._capi" in sys.modules}


def spawn_ranks(script, argv, n, poll_s=0.2, check_parent=True):
    """Run `python script argv` as ranks 0..n-1 of one job on this node; wait for all.
    When a rank fails, the others are terminated (their exact PIDs) and its code returned.
    check_parent=False only for tests that spawn GPU-free scripts from a torch process."""
    state = parent_state()
    if check_parent and (state["cuda_initialized"] or state["hip_runtime_mapped"]):
        raise RuntimeError(f"refusing to spawn ranks from a process that touched the GPU: {state}")
    if os.environ.get(DRYRUN_ENV):
        print(json.dumps({"launcher_parent": state}), flush=True)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env[LAUNCHER_ENV] = "self-spawned"
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    rc = 0
    try:
        alive = list(procs)
        while alive:
            for p in list(alive):
                code = p.poll()
                if code is None:
                    continue
                alive.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in alive:
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def requested_gpus(argv, flag="--gpus"):
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument(flag, type=int, default=1)
    ns, _ = p.parse_known_args(argv)
    return getattr(ns, flag.lstrip("-").replace("-", "_"))


def maybe_spawn(script, argv=None, flag="--gpus"):
    """Called by an entry point before it imports torch.  With `flag` N > 1 and no external
    launcher (WORLD_SIZE unset), spawn N ranks of `script` and exit with their code; else
    return (this process is a rank, or the only one)."""
    argv = sys.argv[1:] if argv is None else argv
    if "WORLD_SIZE" in os.environ:
        if os.environ.get(DRYRUN_ENV):
            keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", LAUNCHER_ENV)
            print(json.dumps({"rank_env": {k: os.environ.get(k) for k in keys}}), flush=True)
            sys.exit(0)
        return
    n = requested_gpus(argv, flag)
    if n > 1:
        sys.exit(spawn_ranks(script, argv, n))

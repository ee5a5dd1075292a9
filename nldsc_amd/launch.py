"""One process per GPU, started from a plain `python bench.py --gpus N` (or `python -m nldsc_amd ... --gpus N`).

The driver may start the ranks itself (`torch.distributed.run --nproc-per-node N bench.py --gpus N`); when it
does not, `WORLD_SIZE` is unset and the parent process starts `torch.distributed.run` as a CHILD process with the
same arguments (never an exec: nothing in the parent has touched the GPU, and it only waits for the child), so the
N ranks run exactly as they would under the driver's launcher: one rank per GPU, RCCL over xGMI, rendezvous on
127.0.0.1.  The ranks' stdout is inherited, so rank 0's one JSON line is the parent's output; the parent exits
with the child's status.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import Sequence


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_devices() -> int:
    """HIP devices this process could use, counted without initialising the GPU (torch.cuda.device_count()
    reads the device list; it does not create a HIP context on this image)."""
    import torch
    return int(torch.cuda.device_count())


def spawn_ranks(script: str, argv: Sequence[str], n: int, *, env: dict | None = None,
                timeout: float | None = None) -> int:
    """Run `script argv` as n ranks under torch.distributed.run in a child process; returns its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script] + list(argv)
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL across processes)
    try:
        return subprocess.run(cmd, env=e, timeout=timeout).returncode
    except subprocess.TimeoutExpired:
        return 124


def ranks_or_spawn(script: str, argv: Sequence[str], gpus: int, backend: str) -> int | None:
    """Called first thing by a multi-GPU entry point.  Returns None when this process is a rank (or a single-GPU
    run) and should go on; otherwise the exit code of the N ranks it started.  Raises SystemExit when the request
    cannot be honoured: a rank count that differs from --gpus, or fewer devices than --gpus for RCCL."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}: launch as many ranks as --gpus")
        return None
    if gpus <= 1:
        return None
    if backend == "nccl":
        n = visible_devices()
        if n < gpus:
            raise SystemExit(f"--gpus {gpus}: only {n} HIP devices visible (one rank per GPU over RCCL; "
                             f"--backend gloo rehearses several ranks on one GPU)")
    return spawn_ranks(script, argv, gpus)

"""Single-node multi-rank launcher of the batched GP-MPC path (one process per GPU).

``bench.py --gpus N`` (and any script using :func:`maybe_spawn`) started WITHOUT torchrun
re-runs itself as ``python -m torch.distributed.run --nnodes 1 --nproc-per-node N
--master-addr 127.0.0.1`` in a CHILD process and exits with its return code.  This happens
before the parent touches the GPU (no HIP call, no ``torch.cuda`` query), so the parent never
holds a device context and never replaces itself (no exec).  Under torchrun (``WORLD_SIZE``
set) nothing is spawned.  Ranks read RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the env.

``GPMPC_DIST_BACKEND`` selects the process-group backend: ``nccl`` (= RCCL over xGMI on ROCm,
the default on GPUs) or ``gloo`` (CPU rehearsal of the multi-rank path, used by the CPU tests).
"""

from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def needs_spawn(nprocs: int) -> bool:
    """True when N > 1 ranks were asked for but this process was not started by torchrun."""
    return nprocs > 1 and "WORLD_SIZE" not in os.environ


def spawn(nprocs: int, script: str, argv: list[str], env: dict | None = None) -> int:
    """Run ``script argv`` as ``nprocs`` ranks under torch.distributed.run (child process)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nprocs),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), script, *argv]
    e = dict(os.environ if env is None else env)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL on this host driver
    return subprocess.call(cmd, env=e)


def maybe_spawn(nprocs: int, script: str, argv: list[str]) -> None:
    """If needed, launch ``nprocs`` ranks of ``script`` and exit this process with their code."""
    if needs_spawn(nprocs):
        sys.exit(spawn(nprocs, script, argv))


def rank_env() -> tuple[int, int, int]:
    """(rank, local_rank, world_size) from the torchrun environment (1 rank without it)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))

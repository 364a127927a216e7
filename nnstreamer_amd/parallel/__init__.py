"""Multi-GPU helpers: one process per GPU (torchrun-style), branch data
parallelism and rank groups.

The reference has no collectives: stream-level data
parallelism is built by hand from tee / tensor_demux branches, and tensors
cross processes only through tensor_query / edge sockets.  nnsx keeps that
model and maps it onto MI355X nodes:

* every rank runs its own pipeline pinned to GPU ``LOCAL_RANK``
  (:func:`rank_info`, :func:`format_pipeline`) -- "branch-DP";
* rank-to-rank traffic uses the connect-type=RCCL edge / query elements and
  ``tensor_allgather`` (RCCL over xGMI, control plane on a TCP store at
  ``MASTER_ADDR:MASTER_PORT+17``), see csrc/comm/group.h;
* :func:`gather_stats` folds per-rank measurements (max / sum) over the
  default ``torch.distributed`` process group (RCCL or gloo).

Launch like any torch job::

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 app.py
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class RankInfo:
    rank: int
    world: int
    local_rank: int
    device: int  # GPU of this rank, -1 on a host without GPUs
    store: str   # control-plane store host:port of the rank groups

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def rank_info(use_gpu: bool = True) -> RankInfo:
    """Rank / world / device of this process from the torchrun environment."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    dev = -1
    if use_gpu:
        from .. import gpu_count

        n = gpu_count()
        dev = local % n if n > 0 else -1
    store = os.environ.get("NNSX_STORE", "")
    if not store:
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29570"))
        store = f"{addr}:{port + 17}"
    return RankInfo(rank, world, local, dev, store)


def format_pipeline(template: str, info: RankInfo | None = None, **extra) -> str:
    """Fill ``{rank}``, ``{world}``, ``{local_rank}``, ``{device}`` and
    ``{store}`` (plus ``extra``) into a launch description, e.g.
    ``"... ! tensor_filter device={device} ! tensor_allgather store={store} ! ..."``."""
    info = info or rank_info()
    return template.format(rank=info.rank, world=info.world, local_rank=info.local_rank, device=info.device,
                           store=info.store, **extra)


def split_work(n_items: int, info: RankInfo | None = None) -> range:
    """Contiguous share of ``n_items`` for this rank."""
    info = info or rank_info(use_gpu=False)
    per, rem = divmod(n_items, info.world)
    start = info.rank * per + min(info.rank, rem)
    return range(start, start + per + (1 if info.rank < rem else 0))


def gather_stats(values, op: str = "max"):
    """Reduce a list of floats over the default process group (no-op when
    torch.distributed is not initialised).  op: "max" | "sum" | "min"."""
    import torch

    vals = [float(v) for v in values]
    try:
        import torch.distributed as dist

        if not (dist.is_available() and dist.is_initialized()):
            return vals
    except Exception:  # noqa: BLE001
        return vals
    t = torch.tensor(vals, dtype=torch.float64)
    if dist.get_backend() == "nccl":
        t = t.cuda()
    red = {"max": dist.ReduceOp.MAX, "sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN}[op]
    dist.all_reduce(t, op=red)
    return t.cpu().tolist()


__all__ = ["RankInfo", "rank_info", "format_pipeline", "split_work", "gather_stats"]

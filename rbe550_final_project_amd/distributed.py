"""Rank group for the data-parallel planner: one process per GPU.

Each RRT-Connect iteration shards its samples across the ranks (rank r takes
samples [r * B/world, (r + 1) * B/world) of the global Philox stream); every rank
runs nearest-node search, steering, the extension edge and the connect chain of
its slice on its GPU, then ONE all-gather per iteration exchanges a 12-byte record
per sample (accepted extension's nearest node or -1, the other tree's nearest node,
valid chain steps | reached) so every rank appends the same nodes in global sample
order: the replicated trees stay bit-identical and the plan equals the world-1
plan (DESIGN.md §4 "Multi-GPU").

Transports (inside librbe_mi355x.so):
  rccl  ncclAllGather on the planner's stream over xGMI; the group's id is made by
        rank 0 and broadcast with torch.distributed (backend "nccl" = RCCL).
  host  the records pass through pinned host buffers and a torch.distributed
        all-gather on CPU tensors (backend "gloo"): ranks sharing one GPU, CPU
        rehearsals.
"""
import torch
import torch.distributed as dist

from . import native


class Group:
    def __init__(self, ctx, transport=None):
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        if transport is None:
            transport = "rccl" if dist.get_backend() == "nccl" else "host"
        if transport not in ("rccl", "host"):
            raise ValueError(f"unknown transport {transport!r}")
        self.transport = transport
        self.calls = 0
        self.ctx = ctx
        if transport == "rccl":
            obj = [native.rccl_unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx.group_init_rccl(self.rank, self.world, obj[0])
        else:
            def allgather(send, recv):
                self.calls += 1
                dist.all_gather_into_tensor(torch.from_numpy(recv), torch.from_numpy(send))
            ctx.group_init(self.rank, self.world, allgather)

    def leave(self):
        """Back to single-rank planning on this context."""
        self.ctx.group_leave()

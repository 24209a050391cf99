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
  shm   ranks of one node: a POSIX shared-memory segment (made by rank 0, its
        name broadcast with torch.distributed) that every rank maps; the kernels
        write and read the records in it in place and the ranks meet at a spin
        barrier in it — no copies, no collective call. The default with gloo
        when every rank is on one host ("host" otherwise).
  host  the records pass through pinned host buffers and a torch.distributed
        all-gather on CPU tensors (backend "gloo").
"""
import ctypes
import torch
import torch.distributed as dist

from . import native


SHM_BYTES = 64 << 20   # records of 2 x 2.7M samples at world 2: room for C4 / C5 batches


class Group:
    def __init__(self, ctx, transport=None, shm_bytes=SHM_BYTES):
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        if transport is None:
            if dist.get_backend() == "nccl":
                transport = "rccl"
            else:   # the shared-memory segment exists only on rank 0's host
                import socket
                hosts = [None] * self.world
                dist.all_gather_object(hosts, socket.gethostname())
                transport = "shm" if len(set(hosts)) == 1 else "host"
        if transport not in ("rccl", "host", "shm"):
            raise ValueError(f"unknown transport {transport!r}")
        self.transport = transport
        self.calls = 0
        self.ctx = ctx
        self.shm = None
        if transport == "shm":
            from multiprocessing import shared_memory
            if self.rank == 0:
                self.shm = shared_memory.SharedMemory(create=True, size=shm_bytes)
            obj = [self.shm.name if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            if self.rank != 0:
                self.shm = shared_memory.SharedMemory(name=obj[0])
                try:   # only the creator unlinks (Python 3.10 registers attachers too)
                    from multiprocessing import resource_tracker
                    resource_tracker.unregister(self.shm._name, "shared_memory")
                except Exception:
                    pass
            dist.barrier()
            addr = ctypes.addressof(ctypes.c_char.from_buffer(self.shm.buf))
            ctx.group_init_shm(self.rank, self.world, addr, self.shm.size)
            dist.barrier()
        elif transport == "rccl":
            obj = [native.rccl_unique_id() if self.rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            ctx.group_init_rccl(self.rank, self.world, obj[0])
        else:
            def allgather(send, recv):
                self.calls += 1
                dist.all_gather_into_tensor(torch.from_numpy(recv), torch.from_numpy(send))
            ctx.group_init(self.rank, self.world, allgather)

    def leave(self):
        """Back to single-rank planning on this context (releases the segment)."""
        self.ctx.group_leave()
        if self.shm is not None:
            shm, self.shm = self.shm, None
            shm.close()
            if self.rank == 0:
                shm.unlink()

"""Rank group for the data-parallel planner: one process per GPU, torch.distributed
over RCCL (backend "nccl") on xGMI.

Each RRT-Connect iteration shards its samples (and then its connect targets) across
the ranks; the per-sample results — one int32 (nearest node or -1) per sample, two
int32 (nearest node, valid steps) per connect target — are all-gathered so every
rank appends the same nodes in global sample order and the replicated trees stay
bit-identical. Messages are small (4 B per sample): the exchange
is latency-bound, one all-gather per phase.
"""
import torch
import torch.distributed as dist


class Group:
    def __init__(self, ctx, batch, device):
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        per = (batch + self.world - 1) // self.world
        self.cap = 8 * (per + 4)
        dev = torch.device("cuda", device)
        self.send = torch.zeros(self.cap, dtype=torch.uint8, device=dev)
        self.recv = torch.zeros(self.cap * self.world, dtype=torch.uint8, device=dev)
        self.calls = 0

        staged = dist.get_backend() != "nccl"   # gloo: exchange through host memory

        def allgather(nbytes):
            self.calls += 1
            if staged:
                out = torch.empty(nbytes * self.world, dtype=torch.uint8)
                dist.all_gather_into_tensor(out, self.send[:nbytes].cpu())
                self.recv[: nbytes * self.world].copy_(out)
            else:
                dist.all_gather_into_tensor(self.recv[: nbytes * self.world], self.send[:nbytes])
            torch.cuda.synchronize(dev)

        ctx.group_init(self.rank, self.world, self.send.data_ptr(), self.recv.data_ptr(), self.cap, allgather)
        self.ctx = ctx

    def leave(self):
        """Back to single-rank planning on this context."""
        self.ctx.group_init(0, 1, 0, 0, 0, None)

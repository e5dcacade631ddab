"""CPU stand-ins for the job's RCCL communicator, over a torch.distributed gloo process group.

Test infrastructure only: the product path (meteorgpu.launch.Group) is torch-free and talks
RCCL through libmsdsp; these give the multi-process CPU tests (world size 2 over gloo) the
same two operations -- the allgather of meteorgpu.stream's protocol and the per-hour count
sum of meteorgpu.shard."""
import numpy as np


class TorchComm:
    """torch.distributed process group (gloo on the host; tests and CPU runs)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)

    def allgather(self, a: np.ndarray) -> list[np.ndarray]:
        import torch
        a = np.ascontiguousarray(a)
        n = torch.tensor([a.size], dtype=torch.int64)
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(self.world)]
        self.dist.all_gather(ns, n, group=self.group)
        m = max(int(t.item()) for t in ns)
        buf = np.zeros(max(m, 1), a.dtype)
        buf[: a.size] = a
        t = torch.from_numpy(buf)
        outs = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        return [o.numpy()[: int(k.item())].copy() for o, k in zip(outs, ns)]

    def allgather_fixed(self, a: np.ndarray) -> list[np.ndarray]:
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a).copy())
        outs = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        return [o.numpy().copy() for o in outs]


def allreduce_counts(counts: np.ndarray, group=None) -> np.ndarray:
    """Sum an int64 count vector over the ranks of a torch.distributed process group
    (gloo on the host; the GPU path all-reduces the device histogram with RCCL instead).
    Returns the reduced copy; a no-op without an initialised process group."""
    import torch
    import torch.distributed as dist

    a = np.ascontiguousarray(counts, dtype=np.int64)
    if not (dist.is_available() and dist.is_initialized()):
        return a.copy()
    t = torch.from_numpy(a.copy())
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.numpy()

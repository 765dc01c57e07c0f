"""Helpers of the gloo CPU tests: the pj_comm callbacks over torch.distributed are
paralleljohnson_amd.partition.TorchDistTransport (host buffers); gather_blocks collects
every rank's distance slice. Test infrastructure only; the product transports are RCCL and
the in-process device copies (comm.cpp)."""
import numpy as np
import torch
import torch.distributed as dist

from paralleljohnson_amd.partition import TorchDistTransport as GlooTransport  # noqa: F401


def gather_blocks(local, block, world, n):
    """Every rank's int32 slice (padded to `block` with INF) -> the whole vector on every rank."""
    buf = torch.full((block,), 100000, dtype=torch.int32)
    buf[: len(local)] = torch.from_numpy(np.asarray(local, np.int32))
    out = torch.empty(block * world, dtype=torch.int32)
    dist.all_gather_into_tensor(out, buf)
    return out.numpy()[:n]

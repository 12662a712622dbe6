"""One-process-per-GPU sharding of the attached-vertex routing table.

* Sources (table rows) are split into `world` contiguous shards of ceil(A / world) rows; rank r
  builds rows [r*R, min(A, (r+1)*R)) with the HIP SSSP / pair kernel into its own HBM shard.
* Exchange 1: all-gather of the {f64 lat, f64 rel} rows and of the u16 hop rows (RCCL over xGMI
  on the GPU; any torch.distributed backend works), so every GPU holds the whole A x A table
  for its share of the packet batch.
* Exchange 2: all-reduce(MIN) of the per-rank row minima = the global minimum latency that sets
  the conservative runahead (shd-master.c:98-124; topology_getMinimumLatency).
* Packet routes need no exchange: each rank routes a contiguous P / world slice of the window.

The row builder is injectable only so the gloo CPU tests can stand in for the GPU; the product
default is the HIP library (`Topology.build_rows_into`), and it raises if the library is absent.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist


def rows_per_rank(A: int, world: int) -> int:
    return max(1, math.ceil(A / world)) if A > 0 else 0


def shard_range(A: int, rank: int, world: int):
    R = rows_per_rank(A, world)
    r0 = min(A, rank * R)
    r1 = min(A, r0 + R)
    return r0, r1


def packet_range(P: int, rank: int, world: int):
    per = math.ceil(P / world) if P else 0
    p0 = min(P, rank * per)
    return p0, min(P, p0 + per)


def _all_gather(out: torch.Tensor, shard: torch.Tensor, group=None):
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, shard, group=group)
    else:  # gloo: list form
        world = dist.get_world_size(group)
        parts = list(out.chunk(world, dim=0))
        dist.all_gather(parts, shard, group=group)


class ShardedTable:
    """Owns the rank's shard buffers and the assembled table (all in the rank's device memory)."""

    def __init__(self, A: int, rank: int, world: int, device, group=None):
        self.A, self.rank, self.world, self.group = A, rank, world, group
        self.R = rows_per_rank(A, world)
        self.r0, self.r1 = shard_range(A, rank, world)
        self.device = torch.device(device)
        R = self.R
        # the shard is a view of the rank's slice of the full buffers when world == 1
        self.full_lr = torch.empty((R * world, A, 2), dtype=torch.float64, device=self.device)
        self.full_hops = torch.empty((R * world, A), dtype=torch.int16, device=self.device)
        if world == 1:
            self.lr = self.full_lr
            self.hops = self.full_hops
        else:
            self.lr = torch.empty((R, A, 2), dtype=torch.float64, device=self.device)
            self.hops = torch.empty((R, A), dtype=torch.int16, device=self.device)
        self.rowmin = torch.full((R,), float("inf"), dtype=torch.float64, device=self.device)
        self.gmin = torch.full((1,), float("inf"), dtype=torch.float64, device=self.device)

    def build(self, builder):
        """builder(row0, row1, lr_view, hops_view, rowmin_view) fills this rank's rows."""
        n = self.r1 - self.r0
        if n < self.R:  # padding rows of the last shard
            self.lr[n:].fill_(-1.0)
            self.hops[n:].zero_()
            self.rowmin[n:].fill_(float("inf"))
        if n > 0:
            builder(self.r0, self.r1, self.lr[:n], self.hops[:n], self.rowmin[:n])

    def exchange(self):
        if self.world > 1:
            _all_gather(self.full_lr, self.lr, self.group)
            # u16 hop rows travel as bytes
            _all_gather(self.full_hops.view(torch.uint8), self.hops.view(torch.uint8), self.group)
        self.gmin.copy_(self.rowmin.min().reshape(1))
        if self.world > 1:
            dist.all_reduce(self.gmin, op=dist.ReduceOp.MIN, group=self.group)

    def table(self):
        return self.full_lr[: self.A], self.full_hops[: self.A]


def hip_builder(top, stream=None):
    """Product row builder: the HIP kernels in libshdtopo.so, on the current torch stream."""
    def build(r0, r1, lr, hops, rowmin):
        s = stream if stream is not None else torch.cuda.current_stream().cuda_stream
        top.build_rows_into(r0, r1, lr, hops, rowmin, stream=s)
    return build


def build_distributed(top, rank, world, device, group=None):
    """Build this rank's rows on the GPU, exchange, and install the table in the library."""
    A = len(top.attached_vertices())
    st = ShardedTable(A, rank, world, device, group)
    st.build(hip_builder(top))
    st.exchange()
    lr, hops = st.table()
    # installed in place: the library reads the gathered buffers (no 1.8 GB copy at C4 size)
    top.bind_table_ref(lr, hops, float(st.gmin.item()),
                       stream=torch.cuda.current_stream().cuda_stream)
    return st

"""Multi-rank sharding on CPU with gloo (world size 2): row shards + all-gather + all-reduce(MIN)
assemble exactly the single-process table; packet slices cover the window exactly once.

The per-rank row builder here is the oracle, injected by the test only (the product builder is
the HIP library, shadow_amd.sharding.hip_builder)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import oracle
    from shadow_amd import sharding

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    z = np.load(os.path.join(GOLDEN, "synth_real.npz"))
    g = oracle.OGraph(int(z["V"]), z["eu"], z["ev"], z["elat"], z["eloss"], z["vloss"])
    attached = np.arange(1400, 1437, dtype=np.int32)   # A = 37: uneven shards
    A = len(attached)

    def builder(r0, r1, lr, hops, rowmin):
        lat, rel, hp = g.source_rows(attached[r0:r1], attached)
        lr[..., 0] = torch.from_numpy(lat)
        lr[..., 1] = torch.from_numpy(rel)
        hops.copy_(torch.from_numpy(hp.astype(np.int16)))
        rowmin.copy_(torch.from_numpy(lat.min(axis=1)))

    st = sharding.ShardedTable(A, rank, world, "cpu")
    st.build(builder)
    st.exchange()
    lr, hops = st.table()
    p0, p1 = sharding.packet_range(1001, rank, world)
    np.savez(os.path.join(out_dir, "r%d.npz" % rank), lr=lr.numpy(), hops=hops.numpy(),
             gmin=st.gmin.numpy(), r0=st.r0, r1=st.r1, p0=p0, p1=p1)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_table_equals_single_process(world, tmp_path):
    import oracle
    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    z = np.load(os.path.join(GOLDEN, "synth_real.npz"))
    g = oracle.OGraph(int(z["V"]), z["eu"], z["ev"], z["elat"], z["eloss"], z["vloss"])
    attached = np.arange(1400, 1437, dtype=np.int32)
    lat, rel, hp = g.source_rows(attached, attached)
    rows = []
    pk = []
    for r in range(world):
        d = np.load(os.path.join(tmp_path, "r%d.npz" % r))
        assert np.array_equal(d["lr"][..., 0], lat) and np.array_equal(d["lr"][..., 1], rel)
        assert np.array_equal(d["hops"].astype(np.int32), hp)
        assert d["gmin"][0] == lat.min()
        rows.append((int(d["r0"]), int(d["r1"])))
        pk.append((int(d["p0"]), int(d["p1"])))
    # shards partition the rows and the packet window exactly
    assert rows[0][0] == 0 and rows[-1][1] == len(attached)
    assert all(rows[i][1] == rows[i + 1][0] for i in range(world - 1))
    assert pk[0][0] == 0 and pk[-1][1] == 1001
    assert all(pk[i][1] == pk[i + 1][0] for i in range(world - 1))

"""Multi-GPU sharding logic, exercised on CPU with the
gloo backend at world_size 2 (and 3): every buffer is owned by exactly one
rank and the all-gather of output totals yields consistent global offsets.
The data path itself needs no collective."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from async_amd import shard
from oracle import pyoracle as orc
from tests import util


def test_by_index_covers_everything():
    for nbuf in (0, 1, 7, 1 << 20, 1000003):
        for world in (1, 2, 3, 4, 8):
            spans = [shard.by_index(nbuf, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (lo, n), (lo2, _) in zip(spans, spans[1:]):
                assert lo + n == lo2
            assert spans[-1][0] + spans[-1][1] == nbuf
            assert max(n for _, n in spans) - min(n for _, n in spans) <= 1


def test_by_bytes_balances():
    # Zipf-like lengths 64*r (SURVEY.md §8(d) config 5 shape, small)
    import random
    rng = random.Random(0x2F)
    lengths = [64 * rng.choice([1, 1, 1, 2, 3, 5, 16, 300]) for _ in range(5000)]
    for world in (1, 2, 4, 8):
        b = shard.by_bytes(lengths, world)
        assert b[0] == 0 and b[-1] == len(lengths) and b == sorted(b)
        loads = [sum(lengths[b[r]:b[r + 1]]) for r in range(world)]
        assert sum(loads) == sum(lengths)
        assert max(loads) - min(loads) <= 2 * max(lengths)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nbuf, L = 1000, 37
        lo, n = shard.by_index(nbuf, world, rank)
        # each rank "encodes" its buffers (oracle stands in for the device
        # here: this test is about the exchange, not the kernels)
        data = [bytes((i * 31 + j) & 0xFF for j in range(L)) for i in range(lo, lo + n)]
        out = b"".join(orc.encode(d) for d in data)
        off, totals = shard.exchange_totals(len(out))
        q.put((rank, lo, n, off, totals, out))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_exchange(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    totals = res[0][4]
    assert all(r[4] == totals for r in res)
    whole = b"".join(r[5] for r in res)
    for rank, lo, n, off, _, out in res:
        assert off == sum(totals[:rank]) and len(out) == totals[rank]
        assert whole[off:off + len(out)] == out
    want = b"".join(orc.encode(bytes((i * 31 + j) & 0xFF for j in range(37)))
                    for i in range(1000))
    assert whole == want


def test_ranks_for_amortises_the_exchange():
    # 1 GiB round trip on one MI355X ~0.8 ms; a 20 us exchange at 10 %
    # overhead justifies 4 ranks, 8 only from 1.6 ms of work
    assert shard.ranks_for(0.8e-3, 8, 20e-6) == 4
    assert shard.ranks_for(1.6e-3, 8, 20e-6) == 8
    assert shard.ranks_for(100e-3, 8, 20e-6) == 8      # never more than the world
    assert shard.ranks_for(10e-6, 8, 20e-6) == 1       # tiny batches stay on one GPU
    assert shard.ranks_for(0.8e-3, 1, 20e-6) == 1
    assert shard.ranks_for(0.8e-3, 8, 0.0) == 8
    assert shard.ranks_for(0.8e-3, 8, 20e-6, max_overhead=0.05) == 2


def test_single_process_exchange():
    assert shard.exchange_totals(123) == (0, [123])
    assert torch.tensor([1]).sum() == 1


def _bench(*args, env_extra=None):
    import json
    import subprocess
    import sys
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args],
                       capture_output=True, text=True, env=env, timeout=240)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, [json.loads(ln) for ln in lines], p.stderr


def test_bench_self_launches_ranks():
    """`bench.py --gpus 2` with no launcher around it starts
    torch.distributed.run itself (before any GPU call), every rank joins one
    process group of exactly --gpus ranks, and rank 0 prints one line that
    reports the group's size (the launch and group logic only: --dry-run,
    gloo on CPU)."""
    rc, lines, err = _bench("--gpus", "2", "--backend", "gloo", "--dry-run")
    assert rc == 0, err[-2000:]
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == 2
    assert lines[0]["process_group"] == {"backend": "gloo", "world_size": 2}
    assert lines[0]["ranks_seen"] == [0, 1]
    sc = lines[0]["root_scatter"]  # the scatter leg runs over the same group
    assert "error" not in sc and sc["ms"] > 0
    # the scaled legs' multi-rank plans: config 4 strong-scaled over the
    # ranks (the north star's curve) with its exchange, config 5's shares
    curve = lines[0]["scaling_curve"]
    assert curve["leg"] == "batch_cfg4" and curve["scaling"] == "strong"
    assert curve["buffers_per_rank"] == [1 << 19, 1 << 19] and curve["output_offsets_ok"]
    assert curve["cfg3_buffers_per_rank"] == [1 << 15, 1 << 15]
    c5 = lines[0]["cfg5_egress"]["shards"]
    assert sum(c5["messages_per_rank"]) == 16384
    b = c5["bytes_per_rank"]
    assert abs(b[0] - b[1]) <= (1 << 20) and sum(b) == int(util.zipf_lengths().sum())


def test_bench_refuses_a_mismatched_world():
    """A rank whose world differs from --gpus exits non-zero and prints no
    line: `--gpus 8` can never report an n_gpus=1 measurement."""
    rc, lines, _ = _bench("--gpus", "2", "--dry-run", env_extra={"WORLD_SIZE": "1"})
    assert rc != 0 and lines == []


@pytest.mark.parametrize("world,rank", [(8, 3), (2, 1), (3, 1)])
def test_batch_digest_check_on_a_share(world, rank):
    """bench.py's whole-output check of a sharded batch leg (config 3):
    a rank's share of the buffers, filled from the splitmix64 stream at its
    own offset (the seed shifted by the share's first word), encoded, and
    every digested chunk it holds whole compared with
    tests/golden/batch_digests.json; a corrupted byte is caught.  CPU
    tensors stand in for the device ones (the check copies to the host)."""
    import base64

    import numpy as np

    import bench
    lo, nbuf = shard.by_index(1 << 16, world, rank)
    L, E = 4096, 5464
    seed = (0x5EED + (lo * L // 8) * 0x9E3779B97F4A7C15) % (1 << 64)
    x = util.splitmix64(seed, nbuf * L)
    assert (x[:L] == util.splitmix64(0x5EED, (lo + 1) * L)[lo * L:]).all()
    enc = np.frombuffer(b"".join(base64.b64encode(x[i * L:(i + 1) * L].tobytes())
                                 for i in range(nbuf)), np.uint8).copy()
    t_enc = torch.from_numpy(enc)
    got = bench._batch_digest_check("cfg3", lo, nbuf, L, E, None, t_enc, None, 0)
    c = 1 << 13
    whole = (lo + nbuf) // c - (lo + c - 1) // c
    assert got["encode_sha256_ok"] is (True if whole else None)
    assert got["scope"].startswith(f"{whole} chunks")
    if whole:
        b0 = ((lo + c - 1) // c) * c - lo
        enc[b0 * E + 77] ^= 1
        with pytest.raises(SystemExit):
            bench._batch_digest_check("cfg3", lo, nbuf, L, E, None, torch.from_numpy(enc),
                                      None, 0)

"""CPU, world_size 2 and 4 (gloo): bench.py's self-check of the N > 1 exchange leg (exchange_verify) — the
fingerprints of every gathered row against its sender's, the own row byte for byte, and the
exact_self=False mean bit-identical on every rank (Examples/ray_ad.py:188) — driven with the oracle codec
in place of the HIP codec on the argument sets of bench.py's N > 1 legs (exchange_leg's flat C4 exchange,
exchange_bucket_leg's C3-shaped bucket with per-tensor scales), plus a rank whose received row is corrupted:
every rank must then report parity false."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, corrupt, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import bench
        from adfl_amd.exchange import PeerExchange
        from test_exchange_gloo import OracleCodec

        from adfl_amd import ops

        results = []
        # bench.py's two N > 1 legs: exchange_leg's PeerExchange(n, bits=8) (chunks 1, unpacked) and
        # exchange_bucket_leg's PeerExchange(total, bits=8, layout=BucketLayout(256 near-equal tensors)), at
        # small sizes; plus an int4 chunked flat exchange
        base, rem = divmod(70_001, 256)
        lay = ops.BucketLayout([base + (1 if i < rem else 0) for i in range(256)])
        cases = [(4099, 8, False, 1, None), (12345, 4, True, 3, None), (lay.total, 8, False, 1, lay)]
        for numel, bits, packed, chunks, layout in cases:
            kw = dict(packed=packed, chunks=chunks) if layout is None else dict(layout=layout)
            ex = PeerExchange(numel, bits=bits, device=torch.device("cpu"), codec=OracleCodec(), **kw)
            rng = np.random.default_rng(50 + rank)
            x = torch.from_numpy(rng.standard_normal(numel, dtype=np.float32) * np.float32(1e-3))
            if corrupt:
                # the transport "loses" a byte of rank 0's row on rank 1 only: wrap the gather's wait
                orig = ex.encode_and_gather

                def tampered(flat, orig=orig, ex=ex):
                    works = orig(flat)
                    for w in works:
                        w.wait()
                    if rank == 1:
                        ex.gathered[-1][0, 3] ^= 0x40
                    return [None] * len(works)

                ex.encode_and_gather = tampered
            results.append(bench.exchange_verify(ex, x, world))
        q.put((rank, results))
        dist.destroy_process_group()
    except Exception as e:  # surfaced in the parent
        import traceback
        q.put((rank, f"error {e!r}\n{traceback.format_exc()}"))


def _run(corrupt, world=2):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, corrupt, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        assert not isinstance(v, str), v
    return res


@pytest.mark.parametrize("world", [2, 4])
def test_exchange_verify_passes_on_a_clean_exchange(world):
    res = _run(corrupt=False, world=world)
    assert sorted(res) == list(range(world))
    for rank, checks in res.items():
        for c in checks:
            assert c["parity"] and c["own_row_equal"] and c["mean_identical_on_all_ranks"], (rank, c)
            assert c["rows_mismatched"] == []
    # every rank holds the identical exact_self=False mean
    for r in range(1, world):
        assert [c["mean_fingerprint"] for c in res[0]] == [c["mean_fingerprint"] for c in res[r]]


def test_exchange_verify_flags_a_corrupted_row_on_every_rank():
    res = _run(corrupt=True)
    for rank, checks in res.items():
        for c in checks:
            assert c["parity"] is False, (rank, c)       # the verdict is agreed over ranks
    assert all(c["rows_mismatched"] for c in res[1])      # rank 1 names rank 0's row it received
    assert all(not c["rows_mismatched"] for c in res[0])


def test_fingerprint_is_position_sensitive():
    import bench
    a = torch.arange(1000, dtype=torch.int32)
    b = a.clone()
    b[[10, 11]] = b[[11, 10]]
    assert bench.fingerprint(a) == bench.fingerprint(a.clone())
    assert bench.fingerprint(a) != bench.fingerprint(b)
    c = a.clone().view(torch.uint8)
    c[7] ^= 1
    assert bench.fingerprint(a) != bench.fingerprint(c)

"""CPU multi-process test (gloo, world_size 2 and 3 -- 3 splits the rows unevenly) of config C5 token-parallel (SURVEY.md 8e's
exchange-free alternative): ``DenoiseLoop`` (DiffuseLLM::sample, diffuse-llm-rs/src/lib.rs:853-955)
on every rank over ITS token rows of x (``parallel.token_rows``) through replicated layers -- the
linear layers (lib.rs:806-813) and p_sample (:1152-1215) are per token, so no collective -- with
the noise those rows get in the unsharded loop (``noise_rows``), and its rows of K/V in the sharded
phase-aware cache (``HeadParallelKVCacheEntry``: one all_reduce(MAX) of the K/V extremes per
quantization, lib.rs:121-313).  The oracle's restatement is the local GEMM / p_sample / noise /
quantize.  Checked against the same loop unsharded in one process and the oracle's KVCacheEntry:

* every rank's x_{t-1} equals the unsharded loop's rows r0..r1 bit for bit, at every step;
* the width sequence, the phase and each rank's codes and params of both copies are bit-identical
  to the unsharded entry's for the rank's K/V rows.
"""
import os
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
from tests.test_parallel_gloo import OracleLinear  # noqa: E402
from tests.test_parallel_loop_gloo import (D, HD, HEADS, SEQ, SEED, STEPS, OracleKVOps,  # noqa: E402
                                           OracleLoopOps, _cfg, _free_port, _inputs, _unsharded)

def _worker(rank, world, port, outdir):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import __graft_entry__ as g
    d = g.load_package()
    par = d.parallel
    Ws, bs, K, V, x0 = _inputs()
    M = x0.shape[0]
    r0, r1 = par.token_rows(M, world, rank)
    k0, k1 = par.token_rows(SEQ, world, rank)
    layers = [OracleLinear(torch.from_numpy(W), torch.from_numpy(b) if j % 2 else None, 4, 128)
              for j, (W, b) in enumerate(zip(Ws, bs))]
    cfg = _cfg(d)
    kv = par.HeadParallelKVCacheEntry(torch.from_numpy(np.ascontiguousarray(K[:, k0:k1])),
                                      torch.from_numpy(np.ascontiguousarray(V[:, k0:k1])), cfg.prefill_bits,
                                      cfg.decode_bits, ops=OracleKVOps)
    loop = d.DenoiseLoop(layers, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=SEED, kv_cache=kv, ops=OracleLoopOps,
                         device="cpu", noise_rows=(r0, M))
    rec = {"rows": np.array([r0, r1]), "kvrows": np.array([k0, k1])}
    x = torch.from_numpy(np.ascontiguousarray(x0[r0:r1]))
    for i, t in enumerate(range(STEPS - 1, -1, -1)):     # free-running, as the unsharded reference
        loop.kv_step(t, STEPS)
        x = loop.step(x, t, i)
        rec[f"x{i}"] = x.numpy().copy()
        rec[f"phase{i}"] = np.array([kv.is_prefill_phase, kv.decode_quant_bits])
        for tag, q in (("p", kv.prefill_quantized), ("d", kv.decode_quantized)):
            if q is not None:
                rec[f"{tag}k{i}"], rec[f"{tag}kp{i}"] = q.keys.data.numpy().copy(), q.keys.params.numpy().copy()
                rec[f"{tag}v{i}"], rec[f"{tag}vp{i}"] = q.values.data.numpy().copy(), q.values.params.numpy().copy()
    out = loop.sample(torch.from_numpy(np.ascontiguousarray(x0[r0:r1])), STEPS)   # sample() = the same steps
    rec["sample"] = out.numpy().copy()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module", params=[2, 3])
def results(request, tmp_path_factory):
    world = request.param
    out = tmp_path_factory.mktemp(f"tokloop{world}")
    mp.spawn(_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
    return [dict(np.load(out / f"rank{r}.npz")) for r in range(world)]


@pytest.fixture(scope="module")
def unsharded():
    import __graft_entry__ as g
    return _unsharded(g.load_package())


def test_token_rows_partition():
    import __graft_entry__ as g
    par = g.load_package().parallel
    for M, W in ((2048, 8), (12, 2), (10, 4), (7, 3)):
        rows = [par.token_rows(M, W, r) for r in range(W)]
        assert rows[0][0] == 0 and rows[-1][1] == M
        assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))
        assert max(b - a for a, b in rows) - min(b - a for a, b in rows) <= 1
        assert min(b - a for a, b in rows) >= 1


def test_token_rows_refuses_empty_shards():
    """world > M would hand some ranks zero rows (which could not join the KV step's collective):
    refused, as are ranks outside the world."""
    import __graft_entry__ as g
    par = g.load_package().parallel
    for M, W, r in ((3, 4, 0), (0, 1, 0), (8, 2, 2), (8, 2, -1), (8, 0, 0)):
        with pytest.raises(ValueError):
            par.token_rows(M, W, r)
    assert par.token_rows(4, 4, 3) == (3, 4)


def test_token_parallel_steps_bitexact(results, unsharded):
    xs, _ = unsharded
    for i in range(STEPS):
        for r in results:
            r0, r1 = r["rows"]
            assert np.array_equal(r[f"x{i}"], xs[i + 1][r0:r1]), i
    for r in results:
        r0, r1 = r["rows"]
        assert np.array_equal(r["sample"], xs[STEPS][r0:r1])


def test_token_parallel_kv_state_bitexact(results, unsharded):
    from oracle import oracle as orc
    _, states = unsharded
    for i, (pre, dbits, pq, dq) in enumerate(states):
        for r in results:
            assert bool(r[f"phase{i}"][0]) == pre and int(r[f"phase{i}"][1]) == dbits, i
            k0, k1 = r["kvrows"]
            for tag, q, bits in (("p", pq, 8), ("d", dq, dbits)):
                if q is None:
                    assert f"{tag}k{i}" not in r, (i, tag)
                    continue
                for which, (codes, s, z) in (("k", q[0]), ("v", q[1])):
                    full = codes.reshape(1, SEQ, HEADS * HD)[:, k0:k1]
                    mine = orc.unpack_bits(r[f"{tag}{which}{i}"], full.size, bits).reshape(full.shape)
                    assert np.array_equal(mine, full), (i, tag, which)
                    assert np.array_equal(r[f"{tag}{which}p{i}"].view(np.uint32),
                                          np.array([s, z], np.float32).view(np.uint32)), (i, tag, which)

"""CPU multi-process test (gloo, world_size 2) of the head-sharded KV cache of
diffusion-llm-rs_amd/parallel.py: per-shard extremes, one all_reduce(MAX), then
params and codes bit-identical to the unsharded per-tensor quantize_tensor
(diffuse-llm-rs/src/quantization.rs:38-68), and per-head attention equal to the unsharded call.
The local steps are the oracle's restatement (the GPU test of the same class runs the HIP ops)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
S, H, D, BITS, WORLD = 48, 5, 128, 4, 2


class OracleKVOps:
    """HeadParallelKVCache's per-shard steps restated by oracle/oracle_np.py (CPU)."""

    @staticmethod
    def extremes(x):
        from oracle import oracle_np as onp
        a = x.numpy()
        return torch.tensor([onp.fold_min(a), onp.fold_max(a)], dtype=torch.float32)

    @staticmethod
    def params(stats, bits):
        from oracle import oracle_np as onp
        mn, mx = stats.numpy()
        return torch.tensor(onp.params_from_extremes(mx, mn, bits), dtype=torch.float32)

    @staticmethod
    def quantize(x, bits, params):
        from oracle import oracle_np as onp
        s, z = params.numpy()
        return torch.from_numpy(onp.pack_bits(onp.quantize_with_params(x.numpy(), bits, s, z), bits))

    @staticmethod
    def attention(q, k, v):
        from oracle import oracle as orc
        from oracle import oracle_np as onp
        deq = []
        for t in (k, v):
            n = int(np.prod(t.shape))
            codes = onp.unpack_bits(t.data.numpy(), n, t.bits)
            s, z = t.params.numpy()
            deq.append(onp.dequantize_tensor(codes, s, z).reshape(t.shape))
        return torch.from_numpy(orc.attention(q.numpy().astype(np.float32), deq[0], deq[1], nthreads=1))


def _inputs():
    rng = np.random.default_rng(7)
    K = rng.standard_normal((S, H, D)).astype(np.float32)
    V = (rng.standard_normal((S, H, D)) * 3 - 1).astype(np.float32)
    K[3, 4, 5] = np.nan                                   # NaN is skipped by the extremes fold
    V[0, 0, 0] = 9.5                                      # the global max sits on rank 0's heads
    Q = rng.standard_normal((S, H, D)).astype(np.float16).astype(np.float32)
    return Q, K, V


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import __graft_entry__ as g
    par = g.load_package().parallel
    Q, K, V = _inputs()
    kv = par.HeadParallelKVCache(H, BITS, ops=OracleKVOps)
    h0, h1 = kv.h0, kv.h1
    loc = [torch.from_numpy(np.ascontiguousarray(a[:, h0:h1])) for a in (Q, K, V)]
    e = kv.entry(loc[1], loc[2])
    O = kv.attention(loc[0], e)
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), heads=np.array([h0, h1]), kc=e.keys.data.numpy(),
             kp=e.keys.params.numpy(), vc=e.values.data.numpy(), vp=e.values.params.numpy(), O=O.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def kv_results(tmp_path_factory):
    out = tmp_path_factory.mktemp("kvgloo")
    mp.spawn(_worker, args=(WORLD, _free_port(), str(out)), nprocs=WORLD, join=True)
    return [dict(np.load(out / f"rank{r}.npz")) for r in range(WORLD)]


def test_head_shards_quantize_bitexact(kv_results):
    from oracle import oracle_np as onp
    Q, K, V = _inputs()
    assert kv_results[0]["heads"][0] == 0 and kv_results[-1]["heads"][1] == H
    for name, full in (("k", K), ("v", V)):
        q, s, z = onp.quantize_tensor(full, BITS)           # the unsharded per-tensor quantization
        q = q.reshape(S, H, D)
        for r in kv_results:
            h0, h1 = r["heads"]
            assert np.array_equal(r[name + "p"].view(np.uint32), np.array([s, z], np.float32).view(np.uint32))
            codes = onp.unpack_bits(r[name + "c"], S * (h1 - h0) * D, BITS).reshape(S, h1 - h0, D)
            assert np.array_equal(codes, q[:, h0:h1])


def test_head_shards_attention_equals_unsharded(kv_results):
    from oracle import oracle as orc
    from oracle import oracle_np as onp
    Q, K, V = _inputs()
    Kh = onp.dequantize_tensor(*onp.quantize_tensor(K, BITS)).reshape(S, H, D)
    Vh = onp.dequantize_tensor(*onp.quantize_tensor(V, BITS)).reshape(S, H, D)
    O = orc.attention(Q, Kh, Vh, nthreads=1)
    for r in kv_results:
        h0, h1 = r["heads"]
        np.testing.assert_array_equal(r["O"], O[:, h0:h1])

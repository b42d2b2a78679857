"""CPU multi-process test (gloo, world_size 2) of config C5 sharded as a whole loop:
``DenoiseLoop`` (DiffuseLLM::sample, diffuse-llm-rs/src/lib.rs:853-955) over hidden-dim-sharded
``TensorParallelPair`` layers (one all_reduce per pair) with the head-sharded phase-aware
``HeadParallelKVCacheEntry`` (lib.rs:121-313: phase switch, progressive decode widths, one
all_reduce(MAX) of the K/V extremes per quantization, both widths from it) on every rank -- the
code the GPU ranks run, with the oracle's restatement as the local steps (GEMM, p_sample, noise,
quantize).  Checked against the same loop unsharded in one process and the oracle's
KVCacheEntry restatement, at every step:

* x_{t-1} of every rank equals the unsharded loop's within f32 summation order (the pair's partial
  sums are reduced in a different order), and the two ranks hold the same bits;
* the width sequence, the phase and each rank's codes and params of both copies are bit-identical
  to the unsharded entry's for the rank's heads.
"""
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
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
from tests.test_parallel_gloo import OracleLinear  # noqa: E402
from tests.test_parallel_kv_gloo import OracleKVOps as _KVOps  # noqa: E402

M, D, PAIRS, STEPS, SEED = 12, 256, 2, 8, 3
SEQ, HEADS, HD = 10, 4, 16
WORLD = 2


class OracleKVOps(_KVOps):
    @staticmethod
    def quantize_pair(x, bits_a, bits_b, params_a, params_b):
        return _KVOps.quantize(x, bits_a, params_a), _KVOps.quantize(x, bits_b, params_b)

    @staticmethod
    def dequantize(t):
        from oracle import oracle_np as onp
        n = int(np.prod(t.shape))
        s, z = t.params.numpy()
        return torch.from_numpy(onp.dequantize_tensor(onp.unpack_bits(t.data.numpy(), n, t.bits), s, z).reshape(t.shape))


class OracleLoopOps:
    """DenoiseLoop's elementwise steps restated by the C oracle (p_sample of lib.rs:1152-1215 over x
    as one sample, the seeded noise stream)."""

    @staticmethod
    def p_sample(x, eps, noise, coef, flag, seed, offset, out):
        from oracle import oracle as orc
        n = x.numel()
        nz = (noise.numpy() if noise is not None else orc.randn(seed, offset, n)).reshape(1, n)
        y = orc.p_sample(x.numpy().reshape(1, n), eps.numpy().reshape(1, n), nz, coef.numpy(), add_noise=flag)
        out.copy_(torch.from_numpy(y.reshape(tuple(x.shape))))

    @staticmethod
    def randn(out, seed, offset):
        from oracle import oracle as orc
        out.copy_(torch.from_numpy(orc.randn(seed, offset, out.numel()).reshape(tuple(out.shape))))


def _inputs():
    rng = np.random.default_rng(11)
    Ws = [(rng.standard_normal((D, D)) / np.sqrt(D)).astype(np.float32) for _ in range(2 * PAIRS)]
    bs = [(0.05 * rng.standard_normal(D)).astype(np.float32) for _ in range(2 * PAIRS)]
    K = (rng.standard_normal((1, SEQ, HEADS * HD)) * 2 + 0.3).astype(np.float32)
    V = rng.standard_normal((1, SEQ, HEADS * HD)).astype(np.float32)
    V[0, 3, 5] = 7.5                      # the global max of V on rank 0's heads
    K[0, 7, HEADS * HD - 2] = -9.0        # the global min of K on rank 1's heads
    x0 = rng.standard_normal((M, D)).astype(np.float32)
    return Ws, bs, K, V, x0


def _cfg(d):
    return d.DiffusionConfig(num_timesteps=STEPS, hidden_size=D, num_layers=2 * PAIRS, num_attention_heads=HEADS)


def _run(d, layers, kv, teacher):
    """The loop step by step (teacher-forced: every step maps the SAME x_t, the unsharded run's),
    recording x_{t-1} and the cache state after each step."""
    cfg = _cfg(d)
    loop = d.DenoiseLoop(layers, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=SEED, kv_cache=kv, ops=OracleLoopOps,
                         device="cpu")
    rec = {}
    x = torch.from_numpy(teacher[0])
    for i, t in enumerate(range(STEPS - 1, -1, -1)):
        loop.kv_step(t, STEPS)
        y = loop.step(x, t, i)
        rec[f"x{i}"] = y.numpy().copy()
        rec[f"phase{i}"] = np.array([kv.is_prefill_phase, kv.decode_quant_bits])
        for tag, q in (("p", kv.prefill_quantized), ("d", kv.decode_quantized)):
            if q is not None:
                rec[f"{tag}k{i}"], rec[f"{tag}kp{i}"] = q.keys.data.numpy().copy(), q.keys.params.numpy().copy()
                rec[f"{tag}v{i}"], rec[f"{tag}vp{i}"] = q.values.data.numpy().copy(), q.values.params.numpy().copy()
        x = torch.from_numpy(teacher[i + 1]) if teacher is not None and i + 1 < len(teacher) else y
    return rec


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _unsharded(d):
    """The same loop, one process, unsharded layers (A then B per pair, f16 between layers) and
    the oracle's KVCacheEntry; free-running, so its states are the teacher sequence."""
    Ws, bs, K, V, x0 = _inputs()
    layers = [OracleLinear(torch.from_numpy(W), torch.from_numpy(b) if j % 2 else None, 4, 128)
              for j, (W, b) in enumerate(zip(Ws, bs))]
    cfg = _cfg(d)
    loop = d.DenoiseLoop(layers, cfg, cumprod=d.Cumprod.INCLUSIVE, seed=SEED, kv_cache=None, ops=OracleLoopOps,
                         device="cpu")
    from oracle import oracle as orc
    ref = orc.KVCacheEntryRef(K, V, cfg.prefill_bits, cfg.decode_bits)
    xs, states = [x0], []
    x = torch.from_numpy(x0)
    for i, t in enumerate(range(STEPS - 1, -1, -1)):
        orc.sample_kv_step(ref, t, STEPS, cfg.decode_bits, cfg.min_decode_bits)
        states.append((ref.is_prefill_phase, ref.decode_quant_bits, ref.prefill_quantized, ref.decode_quantized))
        x = loop.step(x, t, i)
        xs.append(x.numpy().copy())
    return xs, states


def _worker(rank, world, port, outdir):
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import __graft_entry__ as g
    d = g.load_package()
    par = d.parallel
    Ws, bs, K, V, x0 = _inputs()
    teacher, _ = _unsharded(d)
    pairs = [par.TensorParallelPair(torch.from_numpy(Ws[2 * p]), None, torch.from_numpy(Ws[2 * p + 1]),
                                    torch.from_numpy(bs[2 * p + 1]), 4, 128, local_factory=OracleLinear)
             for p in range(PAIRS)]
    c0, c1 = par.head_columns(HEADS * HD, HEADS, world, rank)
    cfg = _cfg(d)
    kv = par.HeadParallelKVCacheEntry(torch.from_numpy(np.ascontiguousarray(K[..., c0:c1])),
                                      torch.from_numpy(np.ascontiguousarray(V[..., c0:c1])), cfg.prefill_bits,
                                      cfg.decode_bits, ops=OracleKVOps)
    rec = _run(d, pairs, kv, teacher)
    rec["cols"] = np.array([c0, c1])
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **rec)
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def loop_results(tmp_path_factory):
    out = tmp_path_factory.mktemp("loopgloo")
    mp.spawn(_worker, args=(WORLD, _free_port(), str(out)), nprocs=WORLD, join=True)
    return [dict(np.load(out / f"rank{r}.npz")) for r in range(WORLD)]


@pytest.fixture(scope="module")
def unsharded():
    import __graft_entry__ as g
    return _unsharded(g.load_package())


def test_sharded_loop_steps_match_unsharded(loop_results, unsharded):
    xs, _ = unsharded
    for i in range(STEPS):
        ref = xs[i + 1]
        for r in loop_results:
            got = r[f"x{i}"]
            rel = np.linalg.norm(got - ref) / np.linalg.norm(ref)
            assert rel <= 1e-5, (i, rel)
        assert np.array_equal(loop_results[0][f"x{i}"], loop_results[1][f"x{i}"]), i   # replicated state


def test_sharded_kv_state_bitexact(loop_results, unsharded):
    from oracle import oracle as orc
    _, states = unsharded
    n_full = SEQ * HEADS * HD
    widths = []
    for i, (pre, dbits, pq, dq) in enumerate(states):
        widths.append(int(dbits))
        for r in loop_results:
            assert bool(r[f"phase{i}"][0]) == pre and int(r[f"phase{i}"][1]) == dbits, i
            c0, c1 = r["cols"]
            for tag, q, bits in (("p", pq, 8), ("d", dq, dbits)):
                if q is None:
                    assert f"{tag}k{i}" not in r, (i, tag)
                    continue
                for which, (codes, s, z) in (("k", q[0]), ("v", q[1])):
                    full = codes.reshape(1, SEQ, HEADS * HD)[..., c0:c1]
                    n = full.size
                    mine = orc.unpack_bits(r[f"{tag}{which}{i}"], n, bits).reshape(full.shape)
                    assert np.array_equal(mine, full), (i, tag, which)
                    assert np.array_equal(r[f"{tag}{which}p{i}"].view(np.uint32),
                                          np.array([s, z], np.float32).view(np.uint32)), (i, tag, which)
    assert n_full % WORLD == 0
    assert widths[: STEPS // 2 - 1] == [4] * (STEPS // 2 - 1) and widths[-1] == 0, widths


def test_cpu_sample_is_the_step_sequence(unsharded):
    """``DenoiseLoop.sample`` on the CPU (device='cpu' forces the serial schedule and touches no CUDA
    stream) returns the state of the step-by-step loop above, bit for bit."""
    import __graft_entry__ as g
    d = g.load_package()
    xs, _ = unsharded
    Ws, bs, K, V, x0 = _inputs()
    layers = [OracleLinear(torch.from_numpy(W), torch.from_numpy(b) if j % 2 else None, 4, 128)
              for j, (W, b) in enumerate(zip(Ws, bs))]
    loop = d.DenoiseLoop(layers, _cfg(d), cumprod=d.Cumprod.INCLUSIVE, seed=SEED, kv_cache=None, ops=OracleLoopOps,
                         device="cpu")
    out = loop.sample(torch.from_numpy(x0), STEPS)
    assert np.array_equal(out.numpy(), xs[STEPS])

"""CPU multi-process tests (gloo, world_size 2) of the multi-GPU partitioning in
diffusion-llm-rs_amd/parallel.py, with the oracle as the local GEMM: shard quantization is
bit-identical to the unsharded layer, and column/row/pair/token-parallel outputs equal the
unsharded restatement."""
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


class OracleLinear:
    """Local layer for CPU tests: the oracle's a5 restatement (group quantize -> dequant -> f32 GEMM)."""

    def __init__(self, W, bias, bits, group):
        from oracle import oracle as orc
        self.orc = orc
        Wn = W.detach().cpu().numpy().astype(np.float32)
        self.codes, self.scales, self.zps = orc.quantize_weights(Wn, bits, group)
        self.What = orc.dequantize_weights(self.codes, self.scales, self.zps, group)
        self.bias = None if bias is None else bias.detach().cpu().numpy().astype(np.float32)

    def __call__(self, x, out_dtype=torch.float32, out=None):
        X = x.detach().cpu().numpy().astype(np.float32)
        Y = (X.astype(np.float64) @ self.What.astype(np.float64))
        if self.bias is not None:
            Y = Y + self.bias[None, :]
        y = torch.from_numpy(Y.astype(np.float32)).to(out_dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y

    @staticmethod
    def bias_cast(y, bias, out_dtype=torch.float16, out=None):
        """The row-parallel epilogue (bias after the reduction, then the cast), in f32 on the CPU."""
        r = (y if bias is None else y + bias.to(torch.float32)[None, :]).to(out_dtype)
        if out is not None:
            out.copy_(r)
            return out
        return r


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
    par = g.load_package().parallel if hasattr(g.load_package(), "parallel") else None
    if par is None:
        import importlib
        par = importlib.import_module("dllm_amd.parallel")
    rng = np.random.default_rng(0)                       # same full weights on every rank
    K, H, N, M = 512, 768, 384, 24
    WA = torch.from_numpy((0.02 * rng.standard_normal((K, H))).astype(np.float32))
    WB = torch.from_numpy((0.02 * rng.standard_normal((H, N))).astype(np.float32))
    bA = torch.from_numpy((0.1 * rng.standard_normal(H)).astype(np.float32))
    bB = torch.from_numpy((0.1 * rng.standard_normal(N)).astype(np.float32))
    X = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32))
    res = {}
    col = par.ColumnParallelLinear(WA, bA, 4, 128, gather=True, local_factory=OracleLinear)
    res["col_y"] = col(X, out_dtype=torch.float32).numpy()
    res["col_codes"], res["col_range"] = col.local.codes, np.array([col.n0, col.n1])
    # the whole layer on every rank (bench.py's N > 1 value): slice GEMMs + all-gather, unchunked and
    # with the gather of chunk i overlapping chunk i+1's GEMM; and unequal slices (the list gather)
    res["col_gathered"] = col.forward_gathered(X, out_dtype=torch.float32).numpy()
    res["col_gathered_chunked"] = col.forward_gathered(X, out_dtype=torch.float32, chunks=5).numpy()
    col_odd = par.ColumnParallelLinear(WB[:, :352], bB[:352], 4, 128, local_factory=OracleLinear)
    res["col_odd_widths"] = np.array(col_odd._widths())
    res["col_odd_gathered"] = col_odd.forward_gathered(X @ WA, out_dtype=torch.float32, chunks=2).numpy()
    row = par.RowParallelLinear(WA, bA, 4, 128, local_factory=OracleLinear)
    res["row_y"] = row(X, out_dtype=torch.float32).numpy()
    res["row_scales"], res["row_range"] = row.local.scales, np.array([row.k0, row.k1])
    pair = par.TensorParallelPair(WA, bA, WB, bB, 4, 128, local_factory=OracleLinear)
    res["pair_y"] = pair(X, out_dtype=torch.float32).numpy()
    res["pair_y_chunked"] = pair(X, out_dtype=torch.float32, chunks=3).numpy()
    res["row_y_chunked"] = row(X, out_dtype=torch.float32, chunks=5).numpy()
    row_rs = par.RowParallelLinear(WA, bA, 4, 128, local_factory=OracleLinear, reduce="rs_ag")
    res["row_rs_y"] = row_rs(X, out_dtype=torch.float32).numpy()
    res["row_rs_y_odd"] = row_rs(X[:23], out_dtype=torch.float32).numpy()       # padded scatter
    res["row_rs_y_chunked"] = row_rs(X, out_dtype=torch.float32, chunks=3).numpy()
    res["row_rs_y16"] = row_rs(X, out_dtype=torch.float16).float().numpy()
    pair_rs = par.TensorParallelPair(WA, bA, WB, bB, 4, 128, local_factory=OracleLinear, reduce="rs_ag")
    res["pair_rs_y"] = pair_rs(X, out_dtype=torch.float32, chunks=2).numpy()
    tok = par.TokenParallelLinear(WA, bA, 4, 128, local_factory=OracleLinear)
    m0, m1 = tok.token_range(M)
    res["tok_y"], res["tok_range"] = tok(X[m0:m1], out_dtype=torch.float32).numpy(), np.array([m0, m1])
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def gloo_results(tmp_path_factory):
    out = tmp_path_factory.mktemp("gloo")
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    return [dict(np.load(out / f"rank{r}.npz")) for r in range(2)]


def _reference():
    rng = np.random.default_rng(0)
    K, H, N, M = 512, 768, 384, 24
    WA = (0.02 * rng.standard_normal((K, H))).astype(np.float32)
    WB = (0.02 * rng.standard_normal((H, N))).astype(np.float32)
    bA = (0.1 * rng.standard_normal(H)).astype(np.float32)
    bB = (0.1 * rng.standard_normal(N)).astype(np.float32)
    X = rng.standard_normal((M, K)).astype(np.float32)
    return WA, WB, bA, bB, X


def test_shard_quantization_is_bitexact(gloo_results, orc):
    WA, *_ = _reference()
    codes, scales, zps = orc.quantize_weights(WA, 4, 128)
    for r in gloo_results:
        n0, n1 = r["col_range"]
        assert np.array_equal(r["col_codes"], codes[:, n0:n1])
        k0, k1 = r["row_range"]
        assert np.array_equal(r["row_scales"], scales[k0 // 128:k1 // 128])


def test_column_gathered_is_the_whole_layer(gloo_results):
    """forward_gathered (bench.py's N > 1 step) leaves the full [M, N] Y on every rank, equal to the
    unsharded layer, for any token chunking and for unequal column slices."""
    WA, WB, bA, bB, X = _reference()
    Y = OracleLinear(torch.from_numpy(WA), torch.from_numpy(bA), 4, 128)(torch.from_numpy(X)).numpy()
    H = (torch.from_numpy(X) @ torch.from_numpy(WA)).numpy()
    Yb = OracleLinear(torch.from_numpy(WB[:, :352]), torch.from_numpy(bB[:352]), 4, 128)(torch.from_numpy(H)).numpy()
    for r in gloo_results:
        assert r["col_gathered"].shape == Y.shape
        np.testing.assert_allclose(r["col_gathered"], Y, rtol=0, atol=1e-6)
        assert np.array_equal(r["col_gathered_chunked"], r["col_gathered"])
        assert len(set(r["col_odd_widths"].tolist())) == 2          # the list-gather path ran
        np.testing.assert_allclose(r["col_odd_gathered"], Yb, rtol=0, atol=1e-5)
    assert np.array_equal(gloo_results[0]["col_gathered"], gloo_results[1]["col_gathered"])


def test_parallel_outputs_match_unsharded(gloo_results, orc):
    WA, WB, bA, bB, X = _reference()
    lin = OracleLinear(torch.from_numpy(WA), torch.from_numpy(bA), 4, 128)
    Y = lin(torch.from_numpy(X)).numpy()
    for r in gloo_results:
        np.testing.assert_allclose(r["col_y"], Y, rtol=0, atol=1e-6)
        np.testing.assert_allclose(r["row_y"], Y, rtol=0, atol=1e-5)
    # shard ranges tile the index spaces exactly
    assert gloo_results[0]["col_range"][1] == gloo_results[1]["col_range"][0]
    assert gloo_results[0]["row_range"][1] == gloo_results[1]["row_range"][0] and gloo_results[1]["row_range"][1] == 512
    # Megatron pair == unsharded A then B (A output rounded to f16 between layers, as on the GPU)
    Hh = torch.from_numpy(Y).to(torch.float16).to(torch.float32)
    linB = OracleLinear(torch.from_numpy(WB), torch.from_numpy(bB), 4, 128)
    # column shards of A are computed per rank before rounding; the f16 rounding is elementwise,
    # so the pair equals B(f16(A(X))) up to the f32 reduction order of B's partial sums.
    Z = linB(Hh).numpy()
    for r in gloo_results:
        np.testing.assert_allclose(r["pair_y"], Z, rtol=0, atol=2e-5)
    # token replicas: concatenated slices == full output
    ys = [None, None]
    for i, r in enumerate(gloo_results):
        m0, m1 = r["tok_range"]
        np.testing.assert_allclose(r["tok_y"], Y[m0:m1], rtol=0, atol=1e-6)


def test_chunked_allreduce_overlap_is_identical(gloo_results):
    """Row-parallel all-reduce issued per token chunk (async, overlapping the next chunk's GEMM)
    gives the unchunked result bit for bit: rows are independent and a 2-rank sum is order-free."""
    for r in gloo_results:
        assert np.array_equal(r["row_y_chunked"], r["row_y"])
        assert np.array_equal(r["pair_y_chunked"], r["pair_y"])


def test_reduce_scatter_all_gather_mode(gloo_results):
    """reduce="rs_ag" (f32 reduce_scatter over token rows, bias and cast on the local rows, then an
    all_gather of the cast rows) gives the all-reduce result: at world size 2 the f32 sum of two
    partials is order-free, so bit for bit, also with padded (M = 23) and chunked scatters; the
    f16 output is the RNE of the f32 one; the pair equals the all-reduce pair."""
    for r in gloo_results:
        assert np.array_equal(r["row_rs_y"], r["row_y"])
        assert np.array_equal(r["row_rs_y_odd"], r["row_y"][:23])
        assert np.array_equal(r["row_rs_y_chunked"], r["row_y"])
        assert np.array_equal(r["row_rs_y16"], r["row_y"].astype(np.float16).astype(np.float32))
        assert np.array_equal(r["pair_rs_y"], r["pair_y"])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_shard_emulation_partials_sum_to_unsharded(world):
    """``shard=(world, rank)`` (one process, no collective) builds each rank's shard: column
    slices concatenate to the unsharded output exactly, and the row-parallel f32 partials sum to
    it within the f32 reduction-order tolerance -- the composition the GPU tests run on HIP."""
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as g
    par = g.load_package().parallel
    WA, WB, bA, bB, X = _reference()
    lin = OracleLinear(torch.from_numpy(WA), torch.from_numpy(bA), 4, 128)
    Y = lin(torch.from_numpy(X)).numpy()
    Xt = torch.from_numpy(X)
    cols = [par.ColumnParallelLinear(torch.from_numpy(WA), torch.from_numpy(bA), 4, 128, local_factory=OracleLinear,
                                     shard=(world, r)) for r in range(world)]
    assert [c.n0 for c in cols[1:]] == [c.n1 for c in cols[:-1]] and cols[-1].n1 == WA.shape[1]
    np.testing.assert_array_equal(np.concatenate([c(Xt, out_dtype=torch.float32).numpy() for c in cols], 1), Y)
    rows = [par.RowParallelLinear(torch.from_numpy(WA), torch.from_numpy(bA), 4, 128, local_factory=OracleLinear,
                                  shard=(world, r)) for r in range(world)]
    tot = sum(r_.partial(Xt).numpy().astype(np.float64) for r_ in rows) + bA[None, :]
    np.testing.assert_allclose(tot, Y, rtol=0, atol=1e-5)

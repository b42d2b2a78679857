"""DESIGN.md section 6's cost table for config C5 on G = 1/2/4/8 GPUs: per-rank
compute measured in one process (profiles/r05_c5/c5_shard_costs.json, scripts/c5_shard_costs.py)
plus the reduction bytes over a stated xGMI bandwidth.  Prints markdown and writes JSON beside the
input (c5_cost_table.json).

Stated assumptions (not measured here: no multi-GPU box in this round's budget):
* ring all-reduce of B bytes on G ranks moves 2 (G-1)/G B per rank; reduce-scatter and all-gather
  (G-1)/G B each; at a per-rank bandwidth of 153 GB/s (one xGMI link: a single ring) or 700 GB/s
  (RCCL channels over the 7 links at ~65 % of 7 x 153 GB/s);
* the KV step (its HBM-bound quantize of K and V [1, 2048, 4096]) costs 65 us / G per rank plus one
  4-float all_reduce(MAX) priced at 15 us (a small-message RCCL latency); p_sample after an unfused
  sharded pair 17 us (12 B per element of [2048, 4096] at ~6 TB/s); the fused last layer's
  epilogue 20 us / G more than a plain layer.
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "profiles" / "r05_c5" / "c5_shard_costs.json"
M, D = 2048, 4096
KV_US, AR_SMALL_US, PSAMPLE_US, FUSED_EXTRA_US = 65.0, 15.0, 17.0, 20.0
BWS = (153.0, 700.0)   # GB/s per rank


def main(single_gpu_ms=None):
    c = json.loads(SRC.read_text())["G"]
    part = M * D * 4                        # f32 partial of a row-parallel shard
    half = M * D * 2
    rows, out = [], {"assumptions": __doc__.split("Stated assumptions")[1].strip(), "G": {}}
    for G in (1, 2, 4, 8):
        r = c[str(G)]
        kv = KV_US / G + (AR_SMALL_US if G > 1 else 0.0)
        # token-parallel: 12 layers on 2048 / G tokens, fused p_sample, KV rows
        tok = 12 * r["token_parallel_layer_us"] + FUSED_EXTRA_US / G + kv
        e = {"token_parallel_step_us": round(tok, 1)}
        if G == 1:
            e["single_gpu_step_us_model"] = round(tok, 1)
        else:
            comp = 6 * r["pair_compute_us"] + PSAMPLE_US + kv
            e["hidden_dim_compute_only_step_us"] = round(comp, 1)
            for bw in BWS:
                ar = 2 * (G - 1) / G * part / (bw * 1e3)             # us
                rsag = (G - 1) / G * (part + half) / (bw * 1e3)
                e[f"allreduce_per_pair_us@{bw:g}"] = round(ar, 1)
                e[f"rs_ag_per_pair_us@{bw:g}"] = round(rsag, 1)
                e[f"hidden_dim_allreduce_step_us@{bw:g}"] = round(comp + 6 * ar, 1)
                e[f"hidden_dim_rs_ag_step_us@{bw:g}"] = round(comp + 6 * rsag, 1)
                # chunked overlap: each pair's reduction hides under the next chunk's GEMMs at best
                e[f"hidden_dim_rs_ag_overlap_bound_step_us@{bw:g}"] = round(
                    PSAMPLE_US + kv + 6 * max(r["pair_compute_us"], rsag), 1)
        out["G"][G] = e
    base = out["G"][1]["token_parallel_step_us"] if single_gpu_ms is None else single_gpu_ms * 1e3
    out["single_gpu_step_us"] = base
    hdr = ("| G | token-parallel step | speed-up | hidden-dim compute only | hidden-dim rs_ag @153 / @700 GB/s | "
           "allreduce @153 / @700 | rs_ag overlapped (bound) @700 | speed-up (best hidden-dim @700) |")
    print(hdr)
    print("|" + "---|" * 8)
    for G in (1, 2, 4, 8):
        e = out["G"][G]
        t = e["token_parallel_step_us"]
        if G == 1:
            print(f"| 1 | {t:.0f} us | 1.00x | -- | -- | -- | -- | -- |")
            continue
        best = min(e["hidden_dim_rs_ag_overlap_bound_step_us@700"], e["hidden_dim_rs_ag_step_us@700"])
        print(f"| {G} | {t:.0f} us | {base / t:.2f}x | {e['hidden_dim_compute_only_step_us']:.0f} us | "
              f"{e['hidden_dim_rs_ag_step_us@153']:.0f} / {e['hidden_dim_rs_ag_step_us@700']:.0f} us | "
              f"{e['hidden_dim_allreduce_step_us@153']:.0f} / {e['hidden_dim_allreduce_step_us@700']:.0f} us | "
              f"{e['hidden_dim_rs_ag_overlap_bound_step_us@700']:.0f} us | {base / best:.2f}x |")
    (SRC.parent / "c5_cost_table.json").write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main(float(sys.argv[1]) if len(sys.argv) > 1 else None)

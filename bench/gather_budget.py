"""Output all-gather budget of the batch-DP bench: per-rank bytes,
ring vs multi-ring vs direct-mesh transfer time over xGMI, and the overlap headroom against the
measured per-GPU step, for N = 2, 4, 8 ranks of one MI355X node.  Analytical (no 8-GPU node was
available to this build); link and HBM figures are parameters.

Usage: python bench/gather_budget.py [--step-ms 165] [--batch 32] [--link-gbps 153] [--rccl-eff 0.7]
"""
import argparse


def budget(n: int, shard_bytes: float, link: float, hbm_w: float, rccl_eff: float) -> dict:
    recv = (n - 1) * shard_bytes  # bytes every rank receives
    ring1 = recv / link  # one ring: each of the n-1 steps moves one shard over one link
    links = min(n - 1, 7)  # an 8-GPU MI355X node: a full xGMI mesh, 7 links per GPU
    rings = recv / (links * link * rccl_eff)  # RCCL: several rings over different links
    mesh = max(shard_bytes / link, recv / hbm_w)  # one shard per link, all links at once; HBM writes
    return {"n": n, "recv_GB": recv / 1e9, "ring1_ms": ring1 * 1e3, "rccl_multiring_ms": rings * 1e3,
            "mesh_ms": mesh * 1e3}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--step-ms", type=float, default=165.0, help="measured fp32 step at 32 samples per GPU")
    ap.add_argument("--batch", type=int, default=32, help="samples per GPU (weak scaling)")
    ap.add_argument("--link-gbps", type=float, default=153.0, help="one xGMI link, one direction")
    ap.add_argument("--hbm-write-gbps", type=float, default=5000.0)
    ap.add_argument("--rccl-eff", type=float, default=0.7, help="fraction of the links' rate RCCL's rings reach")
    a = ap.parse_args(argv)
    link, hbm = a.link_gbps * 1e9, a.hbm_write_gbps * 1e9
    for dt, es in (("fp32", 4), ("bf16", 2)):
        shard = a.batch * 20 * 720 * 1440 * es
        print(f"# gather dtype {dt}: per-rank output shard {shard / 1e9:.3f} GB "
              f"({a.batch} x 20 x 720 x 1440 x {es} B), step {a.step_ms:.0f} ms")
        print(f"{'N':>2} {'recv GB':>8} {'1 ring ms':>10} {'RCCL rings ms':>14} {'mesh ms':>8} "
              f"{'ring/step':>9} {'rings/step':>10} {'mesh/step':>9}")
        for n in (2, 4, 8):
            b = budget(n, shard, link, hbm, a.rccl_eff)
            print(f"{n:>2} {b['recv_GB']:>8.2f} {b['ring1_ms']:>10.1f} {b['rccl_multiring_ms']:>14.1f} "
                  f"{b['mesh_ms']:>8.1f} {b['ring1_ms'] / a.step_ms:>9.0%} {b['rccl_multiring_ms'] / a.step_ms:>10.0%} "
                  f"{b['mesh_ms'] / a.step_ms:>9.0%}")


if __name__ == "__main__":
    main()

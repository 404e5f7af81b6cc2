"""Headline benchmark (driver contract): FourCastNet AFNO batch-DP inference samples/s on N
MI355X GPUs (one process per GPU, RCCL all-gather of the outputs over xGMI, hipGraph-captured
per-step forward), plus the rfft2 / irfft2 720x1440 fp32 single-op latency (us) and the FNO
SpectralConv2d block (BASELINE config 3) as extra keys.

Metric/config from BASELINE.json: "rfft2 720x1440 us + FourCastNet-FNO samples/sec at 1/2/4/8
MI355X"; FourCastNet AFNO (720x1440, patch 8, embed 768, depth 12, 8 AFNO blocks), batch 32
per GPU (weak scaling), synthetic inputs, random-init weights.

Headline engine = the reference's workflow (/root/reference/README.md:57-75,
/root/reference/tests/test_dft.py:73-115): the FourCastNet model written with the ONNX-contrib
``OnnxRfft2`` / ``OnnxIrfft2`` Functions and stock ops, exported to ONNX (com.microsoft Rfft / Irfft
+ Einsum / LayerNorm / MatMul ...), built into an engine whose build-time graph optimizer maps the
stock patterns onto the hand kernels (every rewrite verified on the device), serialized,
deserialized, and replayed as one hipGraph per step.  The library-native export (com.amd.dft
nodes) is timed as the extra key ``native_export_samples_per_s``.

Headline precision = fp32, the reference's only precision (its plugins accept kFLOAT only,
/root/reference/src/dft_plugins/dft_plugins.cpp:101-102): fp32 activations / residual stream /
spectra / FFTs; GEMMs as 3-product bf16 splits with fp32 accumulation (bf16x3: ~5e-6 relative
error per GEMM, vs ~3e-7 for fp32 FMA and ~1e-3 for TF32).  The bf16 model (bf16 activations,
bf16 MFMA) is reported as ``bf16_samples_per_s``.  Every timed step runs the full forward (all
12 blocks) and the output all-gather; K steps are bracketed by barrier + synchronize, and the
max over ranks is reported.

Scaling modes: weak (default; 32 samples per GPU, the driver's contract) or strong with
``--global-batch G`` (G samples split over the ranks: SURVEY §5.8 sizes the output all-gather for
global B=32 over 8 GPUs).  ``--gather-dtype bf16`` gathers a bf16 copy of an fp32 model's output
(SURVEY §5.8 plan item 3).  On multi-GPU RCCL runs the JSON ``comm_env`` records what RCCL chose
(channels, algorithm / protocol lines from its INIT/TUNING log, parsed by ``rccl_choices``).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype fp32|bf16] [--global-batch G]
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import sys
import tempfile
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import tensorrt_dft_plugins_amd as tdp  # noqa: E402
from tensorrt_dft_plugins_amd.models import AFNOConfig, AFNONet, flops_per_sample  # noqa: E402
from tensorrt_dft_plugins_amd.parallel import DataParallelInference, init_distributed, world_info  # noqa: E402

METRIC = "rfft2 720×1440 µs + FourCastNet-FNO samples/sec at 1/2/4/8 MI355X"
DTYPES = {"fp32": torch.float32, "bf16": torch.bfloat16}
COMM_ENV = ("NCCL_ALGO", "NCCL_PROTO", "NCCL_MIN_NCHANNELS", "NCCL_MAX_NCHANNELS", "RCCL_MSCCL_ENABLE",
            "NCCL_P2P_LEVEL", "MI_DFT_GATHER")


def rccl_choices(text: str) -> dict:
    """What RCCL chose, from its ``NCCL_DEBUG=INFO`` (INIT, TUNING) log: channel counts, the ring
    order, and the algorithm / protocol lines of the tuner (kept verbatim, deduplicated)."""
    out: dict = {}
    m = re.search(r"(\d+) coll channels, (?:(\d+) collnet channels, )?(?:(\d+) nvls channels, )?(\d+) p2p channels", text)
    if m:
        out["coll_channels"] = int(m.group(1))
        out["p2p_channels"] = int(m.group(4))
    rings = re.findall(r"Channel (\d+)/(\d+) :((?: \d+)+)", text)
    if rings:
        out["ring_channels"] = int(rings[0][1])
        out["ring0"] = rings[0][2].strip()
    nr = sorted({int(v) for v in re.findall(r"\bnranks (\d+)", text)})
    if nr:
        out["nranks"] = nr[0] if len(nr) == 1 else nr
    m = re.search(r"[RN]CCL version ([\d.]+\S*)", text)
    if m:
        out["version"] = m.group(1)
    algo = []
    for ln in text.splitlines():
        if re.search(r"\b(algo|Algo|ALGO|proto|Proto|PROTO)\b", ln) and "NCCL_ALGO" not in ln:
            t = re.sub(r"^.*?NCCL INFO\s*", "", ln).strip()
            if t and t not in algo:
                algo.append(t)
    if algo:
        out["tuning"] = algo[:8]
    return out


def _rccl_log_setup(world: int) -> str | None:
    """Point RCCL's INFO log (INIT + TUNING only: nothing per collective) at a per-rank file."""
    if world <= 1 or not os.environ.get("LOCAL_RANK") or os.environ.get("NCCL_DEBUG_FILE"):
        return None
    d = tempfile.mkdtemp(prefix="amd_dft_rccl_")
    os.environ.setdefault("NCCL_DEBUG", "INFO")
    os.environ.setdefault("NCCL_DEBUG_SUBSYS", "INIT,TUNING")
    os.environ["NCCL_DEBUG_FILE"] = os.path.join(d, "rccl.%p.log")
    return d


def _rccl_log_read(d: str | None) -> dict:
    if not d:
        return {}
    text = ""
    for f in glob.glob(os.path.join(d, "rccl.*.log")):
        with open(f, errors="replace") as fh:
            text += fh.read()
    return rccl_choices(text)


def init_single_rank_group() -> None:
    """A process group of one rank (``--force-gather``): RCCL (backend "nccl") on a GPU, Gloo on the
    CPU, rendezvous on 127.0.0.1 and a free port."""
    import socket
    from datetime import timedelta

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    if torch.cuda.is_available():
        dev = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                timeout=timedelta(seconds=300), device_id=dev)
    else:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                timeout=timedelta(seconds=300))


def log(msg: str) -> None:
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def _graph_us(fn, iters: int, rounds: int) -> float:
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1000.0 / iters)
    return round(sorted(ts)[len(ts) // 2], 3)


def time_fft_us(iters: int = 50, rounds: int = 5) -> dict:
    """rfft2 / irfft2 720x1440 fp32 batch 1 (contrib Rfft/Irfft ops), hipGraph of `iters` calls.
    Warm: one input/output reused (both stay in the 256 MB Infinity Cache).  Cold: the calls
    rotate over 80 distinct inputs and outputs (660 MB > the Infinity Cache)."""
    x = torch.randn(1, 720, 1440, device="cuda")
    y = tdp.contrib_rfft(x, signal_ndim=2)
    res = {"rfft2_720x1440_us": _graph_us(lambda: tdp.contrib_rfft(x, signal_ndim=2), iters, rounds),
           "irfft2_720x1440_us": _graph_us(lambda: tdp.contrib_irfft(y, signal_ndim=2), iters, rounds)}
    n = 80
    xs = [torch.randn(1, 720, 1440, device="cuda") for _ in range(n)]
    ys = [tdp.contrib_rfft(t, signal_ndim=2) for t in xs]
    it = {"i": 0}

    def cold_r():
        tdp.contrib_rfft(xs[it["i"] % n], signal_ndim=2)
        it["i"] += 1

    def cold_i():
        tdp.contrib_irfft(ys[it["i"] % n], signal_ndim=2)
        it["i"] += 1

    res["rfft2_720x1440_cold_us"] = _graph_us(cold_r, n, rounds)
    res["irfft2_720x1440_cold_us"] = _graph_us(cold_i, n, rounds)
    return res


def time_fno_block_us(rounds: int = 5) -> dict:
    """BASELINE config 3: FNO SpectralConv2d block, 20 ch, 720x1440, bf16, modes 32x32, batch 1."""
    from tensorrt_dft_plugins_amd.models.fno import FNOBlock

    torch.manual_seed(0)
    blk = FNOBlock(20, 32, 32, backend="amd").cuda().eval()
    x = torch.randn(1, 20, 720, 1440, device="cuda").to(torch.bfloat16)
    with torch.no_grad():
        # the FNO layer (spectral conv + 1x1 conv + GELU, the number tracked since round 1) and the
        # SpectralConv2d alone (rfft2 -> complex mul -> irfft2: config 3's literal definition)
        return {"fno_block_720x1440_bf16_us": _graph_us(lambda: blk(x), 20, rounds),
                "spectral_conv2d_720x1440_bf16_us": _graph_us(lambda: blk.spectral(x), 20, rounds)}


def run_steps(runner, steps: int, warmup: int, world: int, dev, cuda: bool) -> float:
    """Seconds for `steps` timed steps (after `warmup`), max over ranks."""

    def sync():
        if cuda:
            torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(warmup):
        runner.step()
    runner.drain()
    sync()
    barrier()
    sync()
    if getattr(runner, "gather", False) and hasattr(runner, "time_comm"):
        runner.time_comm(True)  # event pair around each timed gather (comm-stream busy time)
    t0 = time.perf_counter()
    for _ in range(steps):
        runner.step()
    runner.drain()
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if cuda else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


class _EngineFn:
    """A deserialized engine's graph as the per-step callable (captured by the DP runner)."""

    def __init__(self, eng):
        self.eng = eng

    def __call__(self, x):
        return self.eng.graph.run(x)[0]


def check_optimizer_report(opt: dict, depth: int, dev) -> None:
    """The contrib engine must have every FourCastNet block on the fused kernels: one ``afno_block``
    rewrite per block and no rejected rewrite (a rejection keeps stock nodes = a slower engine that
    would still run).  Collective on multi-rank runs: if any rank's build falls short, every rank
    exits (no rank left waiting in a collective for one that stopped)."""
    ap = opt.get("applied", {})
    bad = ap.get("afno_block") != depth or bool(opt.get("rejected"))
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([1.0 if bad else 0.0], device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        bad = bool(t.item() > 0)
    if bad:
        raise SystemExit(f"contrib engine not fully optimized on at least one rank: applied {ap}, "
                         f"rejected {opt.get('rejected')}")


def build_runner(cfg, dtype, B, dev, a, seed, input_seed=0, gather_dtype=None, export="contrib"):
    """Model -> ONNX export -> engine build (graph optimizer) -> serialized engine bytes ->
    deserialized engine -> hipGraph-captured DP runner: the timed step is the engine a user
    would load with ``dftexec --loadEngine`` (reference: export -> build -> serialize ->
    deserialize -> execute_v2, /root/reference/tests/test_dft.py:89-115).
    ``export="contrib"``: the reference's way of writing the model (ONNX-contrib Rfft/Irfft + stock
    ops); ``"amd"``: the library-native export (com.amd.dft nodes)."""
    torch.manual_seed(seed)  # the same weights on every rank (data parallel = one model)
    backend = export if dev.type == "cuda" else "amd"  # CPU (harness tests): the model itself
    model = AFNONet(cfg, backend=backend).to(dev).to(dtype).eval()
    torch.manual_seed(seed + 1 + input_seed)  # each rank's own batch
    x = torch.randn(B, cfg.in_chans, *cfg.img_size, device=dev).to(dtype)
    info = {"engine": False}
    fn = model
    if a.engine and dev.type == "cuda":
        from tensorrt_dft_plugins_amd.engine import Engine

        t0 = time.perf_counter()
        built = Engine.build(model, (x,), device=dev, use_graph=False)
        opt = built.header.extra.get("optimizer", {})
        if export == "contrib":
            log(f"{dtype}: contrib graph optimizer: {opt.get('nodes_before')} -> {opt.get('nodes_after')} nodes, "
                f"rewrites {opt.get('applied')}, rejected {opt.get('rejected')} ({opt.get('seconds')} s)")
            check_optimizer_report(opt, cfg.depth, dev)
        blob = built.serialize()
        del built, model
        torch.cuda.empty_cache()
        eng = Engine.deserialize(blob, device=dev, use_graph=False)
        fn = _EngineFn(eng)
        info = {"engine": True, "engine_bytes": len(blob), "engine_build_load_s": round(time.perf_counter() - t0, 1),
                "export": export}
        if export == "contrib":
            info["optimizer"] = {"nodes_before": opt.get("nodes_before"), "nodes_after": opt.get("nodes_after"),
                                 "applied": opt.get("applied"), "rejected": len(opt.get("rejected") or [])}
        log(f"{dtype}: {export} engine exported, serialized ({len(blob) / 1e6:.0f} MB) and deserialized in "
            f"{info['engine_build_load_s']}s")
    t0 = time.perf_counter()
    runner = DataParallelInference(fn, x, gather=not a.no_gather, use_graph=not a.no_graph,
                                   gather_backend=a.gather, gather_dtype=gather_dtype,
                                   force_gather=getattr(a, "force_gather", False))
    log(f"{dtype}: captured forward (graph={runner.cap.use_graph}) in {time.perf_counter() - t0:.1f}s")
    return info, runner


def multi_gpu_diagnostics(runner, steps: int, world: int, dev, cuda: bool) -> dict:
    """Self-checks of a multi-GPU run: the rank count every collective actually spans (an all-reduce
    of ones, which must equal WORLD_SIZE), the comm stream's busy time per timed step (gathers
    only, not their wait for compute) and the cost of one gather with no compute in flight.
    Times are the max over ranks."""
    t = torch.ones(1, device=dev if cuda else "cpu")
    dist.all_reduce(t)
    ranks = int(round(float(t.item())))
    if ranks != world:
        raise SystemExit(f"collective spans {ranks} ranks, WORLD_SIZE is {world}")
    busy = runner.comm_busy_ms()
    # the last timed step's gathered buffer against every rank's local output (exact checksums)
    ver = runner.verify_gather()
    if ver["gather_verified"] is False:
        raise SystemExit(f"gathered output does not match the ranks' local outputs: {ver}")
    g_only = runner.gather_only_ms(5)
    vals = torch.tensor([busy / steps if busy is not None else -1.0, g_only if g_only is not None else -1.0],
                        dtype=torch.float64, device=dev if cuda else "cpu")
    dist.all_reduce(vals, op=dist.ReduceOp.MAX)
    out = {"collective_ranks": ranks, "gather_verified": ver["gather_verified"]}
    if runner.gather_fallback:
        out["gather_fallback"] = runner.gather_fallback
    if vals[0] >= 0:
        out["comm_busy_ms_per_step"] = round(float(vals[0]), 3)
    if vals[1] >= 0:
        out["gather_only_ms"] = round(float(vals[1]), 3)
    return out


def _ensure_library(rank: int, world: int, cuda: bool) -> dict:
    """The benchmarked library must be compiled from exactly these sources ON THIS HOST (the
    reference builds and tests in one command, /root/reference/build_with_docker.sh:39): rebuild
    from source here when the library's embedded digest does not match the sources or when it was
    linked on another host (local rank 0 builds, the others wait).  Recorded in the JSON line."""
    import socket

    from tensorrt_dft_plugins_amd import _build

    st = _build.library_status()
    rebuilt, err = False, None
    if not os.environ.get("MI_DFT_LIB"):
        info = _build.embedded_info(st["path"]) or ""
        other_host = f"host={socket.gethostname()} " not in info + " "
        if (not st["digest_ok"] or (cuda and other_host)) and os.environ.get("MI_DFT_BENCH_BUILD", "1") != "0":
            if int(os.environ.get("LOCAL_RANK", "0")) == 0:
                log("native library " + ("does not match the sources" if not st["digest_ok"] else
                                         "was built on another host") + ": compiling from source here")
                try:
                    _build.build(from_source=True)
                except Exception as e:  # noqa: BLE001 -- keep the shipped library, record why
                    err = str(e)[-300:]
                    log(f"rebuild failed, timing the shipped library: {err}")
            rebuilt = err is None
            if world > 1:
                dist.barrier()
            st = _build.library_status()
    out = {"source_digest_ok": st["digest_ok"], "rebuilt_here": rebuilt}
    if err:
        out["rebuild_error"] = err
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="samples per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="strong scaling: this many samples in total, split over the ranks")
    ap.add_argument("--gather-dtype", choices=["same", "bf16"], default="same",
                    help="dtype of the gathered outputs (bf16: half the xGMI bytes of an fp32 model)")
    ap.add_argument("--depth", type=int, default=12)
    ap.add_argument("--dtype", choices=sorted(DTYPES), default="fp32", help="headline precision")
    ap.add_argument("--extra-steps", type=int, default=10, help="timed steps of the other-precision extra (0: skip)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-engine", dest="engine", action="store_false",
                    help="capture the nn.Module directly instead of the serialized engine")
    ap.add_argument("--export", choices=["contrib", "amd"], default="contrib",
                    help="headline engine: the stock ONNX-contrib export (reference workflow) or the native one")
    ap.add_argument("--native-steps", type=int, default=10,
                    help="timed steps of the native-export fp32 engine extra (0: skip)")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--gather", choices=["rccl", "ipc"], default=os.environ.get("MI_DFT_GATHER", "rccl"),
                    help="output all-gather: RCCL ring collective or direct IPC pushes over xGMI")
    ap.add_argument("--force-gather", action="store_true",
                    help="single process: create a one-rank process group (RCCL on a GPU) and run the output "
                         "all-gather + its verification in every timed step (the multi-GPU comm path on one GPU)")
    ap.add_argument("--no-fft", action="store_true", help="skip the rfft2 720x1440 / FNO block probes")
    ap.add_argument("--tiny", action="store_true", help="tiny model/grid (harness smoke test, CPU ok)")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args(argv)

    rccl_dir = _rccl_log_setup(int(os.environ.get("WORLD_SIZE", "1")))
    rank, world, local = init_distributed()
    if a.force_gather and world == 1 and not dist.is_initialized():
        init_single_rank_group()
    if world != a.gpus and world > 1:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    cuda = torch.cuda.is_available()
    # local % count: lets a Gloo rehearsal (MI_DFT_DIST_BACKEND=gloo) put several ranks on one GPU
    dev = torch.device("cuda", local % torch.cuda.device_count()) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(dev)
    lib_note = _ensure_library(rank, world, cuda)
    tdp.load_plugins()

    if a.tiny:
        cfg = AFNOConfig(img_size=(48, 96), in_chans=4, out_chans=4, embed_dim=64, depth=2, num_blocks=4)
    else:
        cfg = AFNOConfig(depth=a.depth)
    head_dt = DTYPES[a.dtype] if cuda else torch.float32
    if a.global_batch is not None:
        if a.global_batch % world:
            raise SystemExit(f"--global-batch {a.global_batch} is not divisible by {world} ranks")
        B = a.global_batch // world
    else:
        B = a.batch if not a.tiny else min(a.batch, 2)
    gdt = torch.bfloat16 if a.gather_dtype == "bf16" else None

    extra = {}
    if cuda and not a.no_fft and not a.tiny and rank == 0:
        extra.update(time_fft_us())
        extra.update(time_fno_block_us())
        log(f"single-op probes: {extra}")

    head_export = a.export if head_dt == torch.float32 else "amd"  # the contrib model is the reference's fp32
    eng_info, runner = build_runner(cfg, head_dt, B, dev, a, 1234, rank, gather_dtype=gdt, export=head_export)
    log(f"world={world} batch/GPU={B} dtype={head_dt} engine={eng_info.get('export', 'module')}")
    if cuda and a.native_steps > 0 and not a.tiny and head_export == "contrib" and a.engine:
        # the same fp32 model through the library-native export (com.amd.dft nodes), timed before the
        # headline so that neither engine is timed straight after a CPU-only build phase (the GPU
        # clocks down while the ONNX export runs on the host)
        _, r2 = build_runner(cfg, head_dt, B, dev, a, 1234, rank, gather_dtype=gdt, export="amd")
        e2 = run_steps(r2, a.native_steps, 2, world, dev, cuda)
        extra["native_export_samples_per_s"] = round(world * B / (e2 / a.native_steps), 3)
        extra["native_export_ms_per_step"] = round(e2 * 1000.0 / a.native_steps, 3)
        r2.close()
        del r2
        torch.cuda.empty_cache()
    elapsed = run_steps(runner, a.steps, a.warmup, world, dev, cuda)
    gathered = runner.gather
    gather_backend_used = runner.gather_backend
    comm_diag = multi_gpu_diagnostics(runner, a.steps, world, dev, cuda) if gathered else {}
    runner.close()
    del runner
    if cuda:
        torch.cuda.empty_cache()
    ms = elapsed * 1000.0 / a.steps
    samples_per_s = world * B / (elapsed / a.steps)
    tflops = samples_per_s * flops_per_sample(cfg) / 1e12

    if cuda and a.extra_steps > 0 and not a.tiny:
        other = "bf16" if a.dtype == "fp32" else "fp32"
        # same weight / input seeds as the headline: only the precision differs (native export:
        # the contrib model is written the reference's fp32 way)
        _, r2 = build_runner(cfg, DTYPES[other], B, dev, a, 1234, rank, export="amd" if other == "bf16" else a.export)
        e2 = run_steps(r2, a.extra_steps, 2, world, dev, cuda)
        extra[f"{other}_samples_per_s"] = round(world * B / (e2 / a.extra_steps), 3)
        extra[f"{other}_ms_per_step"] = round(e2 * 1000.0 / a.extra_steps, 3)
        if other == "bf16":
            extra["bf16_gelu"] = cfg.bf16_gelu
        r2.close()
        del r2

    rccl = _rccl_log_read(rccl_dir) if rank == 0 else {}
    # the world communicator must span every rank (the all-reduce check above already enforces the
    # collective itself); RCCL may log further, smaller communicators, so this is recorded, not fatal
    if "nranks" in rccl:
        nr = rccl["nranks"] if isinstance(rccl["nranks"], list) else [rccl["nranks"]]
        if world not in nr:
            log(f"warning: RCCL communicators report nranks {nr}, none equals WORLD_SIZE {world}")
            rccl["nranks_mismatch"] = True
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(samples_per_s, 3),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong" if a.global_batch is not None else "weak",
            "vs_baseline": None,
            "dtype": "bf16" if head_dt == torch.bfloat16 else "fp32",
            "data": "synthetic inputs, random-init weights",
            "config": {
                "model": "FourCastNet AFNO (720x1440, patch 8, embed 768, depth %d, 8 AFNO blocks)" % cfg.depth
                if not a.tiny else "tiny AFNO (harness test)",
                "global_batch": world * B,
                "seq_len": cfg.h * cfg.w,
                "parallelism": f"dp{world}",
                "per_gpu_batch": B,
                "hipgraph": not a.no_graph and cuda,
                "runtime": ("serialized engine (stock ONNX-contrib export: com.microsoft Rfft/Irfft + standard ops; "
                            "build-time graph optimizer onto the hand kernels; save/load; hipGraph replay)"
                            if eng_info.get("export") == "contrib" else
                            "serialized engine (ONNX com.amd.dft nodes, save/load, hipGraph replay)")
                if eng_info.get("engine") else "captured nn.Module",
                "engine_bytes": eng_info.get("engine_bytes"),
                **({"optimizer": eng_info["optimizer"]} if "optimizer" in eng_info else {}),
                "output_allgather": gathered,
                "gather_backend": (gather_backend_used if gather_backend_used == "ipc" else
                                   ("rccl" if dist.get_backend() == "nccl" else dist.get_backend()))
                if gathered else None,
                "gemm": "hand-mfma",
                "gemm_precision": "bf16x3 split, fp32 accumulate" if head_dt == torch.float32 else "bf16, fp32 accumulate",
                "gather_dtype": ("bf16" if gdt is not None else ("bf16" if head_dt == torch.bfloat16 else "fp32"))
                if gathered else None,
                "comm_env": dict({k: os.environ[k] for k in COMM_ENV if k in os.environ},
                                 **({"rccl": rccl} if rccl else {})),
            },
            "model_tflops_per_s": round(tflops, 2),
            **({"multi_gpu": dict(comm_diag, **({"rccl_nranks": rccl["nranks"]} if "nranks" in rccl else {}))}
               if comm_diag else {}),
            "library": dict(lib_note, build_info=tdp.build_info()),
        }
        out.update(extra)
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if dist.is_available() and dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())

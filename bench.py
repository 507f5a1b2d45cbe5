#!/usr/bin/env python3
"""ADMM quantized CP factorization benchmark (BASELINE.json metric, config C3).

A step = one ALS sweep of scripts/factorize.py over all 16 resnet18 3x3 convs
(default; `--model resnet50` / `llama7b` run configs C4 / C5)
(4-bit tensor_mseminmax_symmetric, reduction rate 2.0): for each mode A, B, C the
Gram∘Gram / MTTKRP, one batched admm_iteration with max_iter_admm=1000 (999 inner
iterations, eps=0 so no early exit), the re-quantization, then the two
reconstruction errors. Unit: factor-iterations/s (one execution of the loop body
source/admm.py:56-65 on one (layer, mode) factor); 47,952 per step per GPU.

Multi-GPU (one process per GPU, torchrun): every rank factorizes its own resnet18
weight set (replica r: seeds 1000+l+100r) - weak scaling, no data-path collective
- and the converged factors are gathered to rank 0 with one RCCL gather per step.
`--shard layers` instead splits ONE model's layers over the ranks (LPT; strong
scaling, capped by the largest layer - SURVEY §8(e)).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "admm-quantization_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "ADMM iters/sec, resnet18 all conv layers 4-bit r=2.0; rel-Frob err vs CPU ref"
MSE = "tensor_mseminmax_symmetric"
PEAK_F32 = 157.3  # TFLOP/s, MI355X fp32 vector == fp32 MFMA dense peak (MI355X_MICROARCH.md)


def layer_cost(spec, R):
    dims = spec.shape
    return sum(2.0 * d * R * R + 1600.0 * d * R for d in dims)


def lpt(specs, nranks):
    loads = [0.0] * nranks
    owner = {}
    order = sorted(range(len(specs)), key=lambda i: -layer_cost(specs[i], specs[i].rank()))
    for i in order:
        r = min(range(nranks), key=lambda k: loads[k])
        owner[i] = r
        loads[r] += layer_cost(specs[i], specs[i].rank())
    return owner


CONFIG_ID = {"resnet18": "C3", "resnet50": "C4", "llama7b": "C5"}


def workload_name(model, work, max_iter_admm):
    """BASELINE.json config the run measures: C3 resnet18 16 3x3 convs (3-way), C4 resnet50
    48 convs (3x3 -> 3-way, 1x1 -> 2-way), C5 one Llama-7B decoder layer (7 2-way matrices)."""
    n3 = sum(1 for (s, _, _, _) in work if len(s.shape) == 3)
    n2 = len(work) - n3
    kinds = ", ".join(k for k in (f"{n3} 3-way (3x3 conv)" if n3 else "", f"{n2} 2-way" if n2 else "") if k)
    return (f"{CONFIG_ID.get(model, model)}: {model} {len(work)} layers per GPU ({kinds}), 1 ALS sweep x all modes x "
            f"{max_iter_admm - 1} ADMM iters (eps=0), 4-bit mse-minmax, rate 2.0")


def build_workload(model, rank, world, shard, device):
    from admmq import synthetic
    specs = synthetic.MODELS[model]()
    if shard == "layers" and world > 1:
        own = lpt(specs, world)
        mine = [i for i in range(len(specs)) if own[i] == rank]
        replica = 0
    else:
        mine = list(range(len(specs)))
        replica = rank
    work = []
    for i in mine:
        s = specs[i]
        W = torch.from_numpy(synthetic.layer_weight(s, i, replica)).to(device)
        R = s.rank()
        g = torch.Generator().manual_seed(42)
        init = [torch.randn(n, R, generator=g).to(device) for n in s.shape]
        work.append((s, W, R, init))
    return work


def run_step(work, max_iter_admm, num_attempts=200):
    from admmq.factorize import LayerRun, als_sweep
    runs = [LayerRun(s.name, W, R, [f.clone() for f in init]) for (s, W, R, init) in work]
    als_sweep(runs, max_iter_admm, 0.0, 4, MSE, num_attempts=num_attempts)
    return runs


def gather_factors(runs, rank, world, device):
    flat = torch.cat([f.reshape(-1) for r in runs for f in r.factors]) if runs else torch.zeros(0, device=device)
    if world == 1:
        return flat.numel()
    n = torch.tensor([flat.numel()], device=device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    mx = int(max(s.item() for s in sizes))
    buf = torch.zeros(mx, device=device)
    buf[:flat.numel()] = flat
    out = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, out, dst=0)
    return sum(int(s.item()) for s in sizes)


def reduce_over_ranks(elapsed, factor_iters, world, device):
    """Whole-job rate inputs: the slowest rank's elapsed time (MAX) and the
    factor-iterations all ranks processed (SUM)."""
    el = torch.tensor([elapsed], device=device, dtype=torch.float64)
    fi = torch.tensor([float(factor_iters)], device=device, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(fi, op=dist.ReduceOp.SUM)
    return float(el.item()), float(fi.item())


def algorithmic_flops(work, max_iter_admm, num_attempts=200):
    """Per step: SSE sweep 8 flops x candidates x elements (SURVEY §8(d) F_valu) and the
    solve GEMM 2 I R^2, summed over (layer, mode) x inner iterations."""
    it = max_iter_admm - 1
    sse = sum(8.0 * num_attempts * d * R for (s, W, R, _) in work for d in s.shape) * it
    gemm = sum(2.0 * d * R * R for (s, W, R, _) in work for d in s.shape) * it
    return sse, gemm


def gemm_bytes(work):
    """Algorithmic HBM bytes of the solve GEMMs of one ADMM iteration over every mode:
    P and U read, H_T and X = H_T - U written (4 I R floats) and M read (R^2 floats)."""
    return sum(4.0 * (4 * d * R + R * R) for (s, W, R, _) in work for d in s.shape)


TRAFFIC_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01_v9_traffic.json")


def load_traffic():
    """Per-launch HBM bytes of each launch class from the committed rocprofv3 PMC passes
    (tools/traffic_json.py); PMC counters cannot be read live inside the timed region."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
        t["file"] = os.path.relpath(TRAFFIC_FILE, os.path.dirname(os.path.abspath(__file__)))
        return t
    except (OSError, ValueError):
        return None


def cpu_baseline(work, max_iter_admm, sample_iters=20):
    """torch-CPU port of the reference step (oracle/torch_port.py) on a bounded sample:
    every (layer, mode) of the workload, setup + `sample_iters` inner iterations timed,
    extrapolated linearly to max_iter_admm-1 iterations (per-iteration cost is constant
    with eps=0)."""
    from oracle import torch_port
    total = 0.0
    n_fi = 0
    wall = time.time()
    for (s, W, R, init) in work:
        Wc = W.cpu()
        fs = [f.cpu() for f in init]
        for m in range(len(s.shape)):
            G, F = torch_port.gram_mttkrp(Wc, fs, m)
            t0 = time.perf_counter()
            torch_port.admm_iteration(fs[m], torch.zeros_like(fs[m]), F, G, 1, 0.0, 4)
            t1 = time.perf_counter()
            torch_port.admm_iteration(fs[m], torch.zeros_like(fs[m]), F, G, 1 + sample_iters, 0.0, 4)
            t2 = time.perf_counter()
            setup = t1 - t0
            per_iter = max((t2 - t1) - setup, 0.0) / sample_iters
            total += setup + per_iter * (max_iter_admm - 1)
            n_fi += max_iter_admm - 1
    return {"value": n_fi / total, "unit": "factor-iterations/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{len(work)} layers x modes: setup + {sample_iters} inner iterations each timed on host cores "
                      f"(torch-CPU port of source/admm.py + quantization.py, oracle/torch_port.py), extrapolated "
                      f"to {max_iter_admm - 1} iterations; {time.time() - wall:.1f}s of CPU work"}


def parity_check(device):
    """rel-Frob of H_T vs the CPU oracle and bit-exactness of the projection on
    resnet18 layer1.0.conv1 (all modes, one ADMM step)."""
    from oracle import admm_oracle as ao, quant_oracle as qo
    from admmq import synthetic, admm_iteration_batched
    idx, spec = synthetic.find_layer("resnet18", "layer1.0.conv1")
    W = synthetic.layer_weight(spec, idx)
    R = spec.rank()
    g = torch.Generator().manual_seed(42)
    fs = [torch.randn(n, R, generator=g).numpy() for n in W.shape]
    worst = 0.0
    exact = True
    for m in range(3):
        G, F = ao.gram_mttkrp(W, fs, m)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)  # noqa: E731
        (H,), dbg = admm_iteration_batched([(t(fs[m]), torch.zeros(fs[m].shape, device=device), t(F), t(G))], 2, 1e-8,
                                           4, MSE, debug_outputs=True)
        _, _, info = ao.admm_iteration(fs[m], np.zeros_like(fs[m]), F, G, 2, 1e-8, 4, MSE, return_info=True)
        ht = dbg[0][0].cpu().numpy()
        worst = max(worst, float(np.linalg.norm(ht - info["HT"]) / np.linalg.norm(info["HT"])))
        hq = qo.quantize_tensor(dbg[0][1].cpu().numpy(), 4, MSE)
        exact &= bool(np.array_equal(H.cpu().numpy().view(np.uint32), hq.view(np.uint32)))
    return worst, exact


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--max-iter-admm", type=int, default=1000)
    ap.add_argument("--shard", choices=["replica", "layers"], default="replica")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-iters", type=int, default=None,
                    help="inner iterations timed per (layer, mode) on the CPU (default 20; 1 for llama7b)")
    ap.add_argument("--no-profile", action="store_true", help="skip the live HIP-event kernel timing")
    ap.add_argument("--prof-every", type=int, default=16,
                    help="HIP-event timing of one ADMM iteration in N (an event pair per launch adds a gap)")
    ap.add_argument("--exhaustive", action="store_true",
                    help="A/B: evaluate all MSE candidates (reference-style) instead of the two-stage search")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    from admmq import _lib
    lib = _lib.load()
    lib.admmq_set_exhaustive_search(1 if a.exhaustive else 0)
    work = build_workload(a.model, rank, world, a.shard, device)
    fi_per_step = sum(len(s.shape) * (a.max_iter_admm - 1) for (s, _, _, _) in work)

    for _ in range(a.warmup):
        gather_factors(run_step(work, a.max_iter_admm), rank, world, device)
    torch.cuda.synchronize()

    prof = not a.no_profile
    if prof:
        n_launch = a.steps * 3 * 3 * (a.max_iter_admm // a.prof_every + 1) + 64
        _lib.check(lib.admmq_profile_begin(n_launch, a.prof_every), "profile_begin")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        runs = run_step(work, a.max_iter_admm)
        gather_factors(runs, rank, world, device)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern = None
    if prof:
        import ctypes
        ms = (ctypes.c_double * 4)()
        cnt = (ctypes.c_int64 * 4)()
        _lib.check(lib.admmq_profile_end(ms, cnt), "profile_end")
        kern = {"ms": list(ms), "launches": list(cnt)}

    elapsed_max, total_fi = reduce_over_ranks(elapsed, fi_per_step * a.steps, world, device)

    if rank == 0:
        out = {"metric": METRIC, "value": total_fi / elapsed_max, "unit": "factor-iterations/s", "n_gpus": world,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": 1e3 * elapsed_max / a.steps,
               "higher_is_better": True, "scaling": "weak" if a.shard == "replica" else "strong",
               "vs_baseline": None, "dtype": "f32", "data": "synthetic",
               "config": {"workload": workload_name(a.model, work, a.max_iter_admm),
                          "factor_iterations_per_step_per_gpu": fi_per_step, "max_iter_admm": a.max_iter_admm,
                          "parallelism": f"{'replica' if a.shard == 'replica' else 'layer-shard'} x{world}, "
                                         "one RCCL gather of factors per step",
                          "mse_search": "exhaustive" if a.exhaustive else "two-stage exact"}}
        if kern is not None:
            sse_f, gemm_f = algorithmic_flops(work, a.max_iter_admm)
            ms, cnt = kern["ms"], kern["launches"]
            # one ADMM iteration in prof_every is timed, uniformly over the modes, so the
            # class's average launch duration is ms/cnt and its average algorithmic flops
            # per launch is the step's total over all the step's launches
            n_modes = max(len(s.shape) for (s, _, _, _) in work)
            launches_per_step = n_modes * (a.max_iter_admm - 1)
            avg_us = [1e3 * ms[i] / max(cnt[i], 1) for i in range(4)]
            traffic = load_traffic()
            rf = []
            for cls, (flops, bound, name) in enumerate([
                    (gemm_f, "mfma", "k_gemm (solve, MFMA f32)"),
                    (sse_f, "valu", "MSE search (k_mse_hist3: stage 1 + selection + stage 2)")]):
                ach = flops / launches_per_step / (avg_us[cls] * 1e-6) / 1e12 if cnt[cls] else 0.0
                key = ["gemm", "sse"][cls]
                r = {"bound": bound, "achieved": ach, "peak": PEAK_F32, "unit": "TFLOP/s", "frac": ach / PEAK_F32,
                     "traffic": traffic["classes"][key]["bytes_per_launch"] if traffic else None,
                     "traffic_unit": "bytes/launch (HBM, PMC)", "kernel": name,
                     "launch_avg_us": avg_us[cls], "launches_timed": cnt[cls]}
                if traffic:
                    r["traffic_source"] = traffic["file"]
                if cls == 0:
                    r["algorithmic_bytes_per_launch"] = gemm_bytes(work) / n_modes
                rf.append(r)
            dom = max(range(3), key=lambda k: avg_us[k])
            out["roofline"] = rf[1] if dom == 1 else rf[0]
            out["roofline_gemm"] = rf[0]
            out["kernel_ms_per_step"] = {k: avg_us[i] * 1e-3 * (launches_per_step if i < 3 else cnt[3] / a.steps)
                                         for i, k in enumerate(["gemm", "sse", "finalize", "prepare"])}
            out["kernel_avg_us"] = dict(zip(["gemm", "sse", "finalize", "prepare"], avg_us))
            out["prof_every"] = a.prof_every
        if world == 1 and not a.no_cpu_baseline:
            # cpu_baseline leg: the CPU reference port timed on host cores, and the
            # metric's "rel-Frob err vs CPU ref" (oracle comparison of one ADMM step)
            si = a.cpu_sample_iters if a.cpu_sample_iters is not None else (1 if a.model == "llama7b" else 20)
            out["cpu_baseline"] = cpu_baseline(work, a.max_iter_admm, sample_iters=si)
            out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
            try:
                rel, exact = parity_check(device)
                out["rel_frob_vs_cpu_ref"] = rel
                out["projection_bit_exact"] = exact
            except Exception as e:  # parity is reported, never blocks the perf line
                out["parity_error"] = repr(e)[:200]
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""ADMM quantized CP factorization benchmark (BASELINE.json metric, config C3).

A step = one ALS sweep of scripts/factorize.py over all 16 resnet18 3x3 convs
(default; `--model resnet50` / `llama7b` run configs C4 / C5)
(4-bit tensor_mseminmax_symmetric, reduction rate 2.0): for each mode A, B, C the
Gram∘Gram / MTTKRP, one batched admm_iteration with max_iter_admm=1000 (999 inner
iterations, eps=0 so no early exit), the re-quantization, then the two
reconstruction errors. Unit: factor-iterations/s (one execution of the loop body
source/admm.py:56-65 on one (layer, mode) factor); 47,952 per step per GPU.

Multi-GPU (one process per GPU, torchrun): the default `--shard layers`
splits ONE model's layers over the ranks by LPT on layer cost (strong scaling, capped
by the largest layer: the line reports the cap), no data-path collective, and the
converged factors are gathered to rank 0 with one RCCL gather per step. `--shard
replica` instead gives every rank its own weight set (seeds 1000+l+100r, weak scaling).
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


def _model_specs(model):
    from admmq import synthetic
    return synthetic.MODELS[model]()


SHARD_MODEL_FILE = os.path.join(ROOT, "profiles", "r04_shard_model.json")


def measured_cap(model, loads, total):
    """Shard sweep time priced by MEASURED per-sweep time instead of flops: the affine model
    T(shard) = T0 + kappa * cost (cost = the LPT flop model's load) fitted to emulated
    shard timings of this model (tools/fit_shard_model.py -> profiles/r04_shard_model.json;
    T0 is the per-sweep latency floor every shard pays - the thin loop and each inner
    iteration's kernel chain - which the flop model ignores). Returns the implied strong-
    scaling cap T(whole model) / max T(shard) and the fit, or None without a fit."""
    try:
        with open(SHARD_MODEL_FILE) as f:
            fit = json.load(f)[model]
    except (OSError, ValueError, KeyError):
        return None
    t = lambda c: fit["t0_ms"] + fit["kappa_ms_per_cost"] * c  # noqa: E731
    return {"measured_speedup_cap": t(total) / max(t(c) for c in loads),
            "shard_model": {"t0_ms": fit["t0_ms"], "kappa_ms_per_cost": fit["kappa_ms_per_cost"],
                            "source": os.path.relpath(SHARD_MODEL_FILE, ROOT), "fit_max_rel_err": fit["max_rel_err"]}}


def build_workload(model, rank, world, shard, device):
    """This rank's layers (LPT over layer cost when sharding), their
    synthetic weights and seed-42 random init, plus the static shard plan: every rank's
    factor element count (so the final gather needs no size exchange) and the LPT
    load-imbalance cap on the speedup."""
    from admmq import synthetic
    specs = synthetic.MODELS[model]()
    owner = lpt(specs, world) if (shard == "layers" and world > 1) else {i: rank for i in range(len(specs))}
    mine = [i for i in range(len(specs)) if owner[i] == rank]
    replica = rank if shard == "replica" else 0
    work = []
    for i in mine:
        s = specs[i]
        W = torch.from_numpy(synthetic.layer_weight(s, i, replica)).to(device)
        R = s.rank()
        g = torch.Generator().manual_seed(42)
        init = [torch.randn(n, R, generator=g).to(device) for n in s.shape]
        work.append((s, W, R, init))
    numel = [0] * world
    loads = [0.0] * world
    for i, s in enumerate(specs):
        for k in (range(world) if shard == "replica" else [owner[i]]):
            numel[k] += sum(n * s.rank() for n in s.shape)
            loads[k] += layer_cost(s, s.rank())
    total = sum(layer_cost(s, s.rank()) for s in specs)
    info = None
    if shard == "layers":
        info = {"policy": "LPT over whole layers, cost sum_m (2 I_m R^2 + 1600 I_m R) (SURVEY §8(e))",
                "layers_per_rank": [sum(1 for i in owner if owner[i] == k) for k in range(world)],
                "lpt_speedup_cap": total / max(loads),
                "whole_layer_speedup_cap": total / max(layer_cost(s, s.rank()) for s in specs)}
        mc = measured_cap(model, loads, total)
        if mc:
            info.update(mc)
    return work, numel, info


def run_step(work, max_iter_admm, num_attempts=200):
    from admmq.factorize import LayerRun, als_sweep
    runs = [LayerRun(s.name, W, R, [f.clone() for f in init]) for (s, W, R, init) in work]
    als_sweep(runs, max_iter_admm, 0.0, 4, MSE, num_attempts=num_attempts)
    return runs


USE_DIST = False   # torch.distributed (RCCL) on: world > 1, or --force-dist (exercises the collectives at N = 1)


def gather_factors(runs, rank, world, numel, device, keep=None):
    """The single collective of the path: every rank's converged factors to rank 0 (one
    RCCL gather over xGMI). Sizes are static (numel from the shard plan), so the flat
    buffers are padded to the largest rank's size and no size exchange is needed. Returns
    the element count rank 0 holds; `keep` (a list) receives rank 0's per-rank buffers."""
    flat = torch.cat([f.reshape(-1) for r in runs for f in r.factors]) if runs else torch.zeros(0, device=device)
    assert flat.numel() == numel[rank], (flat.numel(), numel[rank])
    if world == 1 and not USE_DIST:
        if keep is not None:
            keep[:] = [flat]
        return flat.numel()
    buf = torch.zeros(max(numel), device=device)
    buf[:flat.numel()] = flat
    out = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, out, dst=0)
    if keep is not None and rank == 0:
        keep[:] = [out[k][:numel[k]] for k in range(world)]
    return sum(numel)


def reduce_over_ranks(elapsed, factor_iters, world, device):
    """Whole-job rate inputs: the slowest rank's elapsed time (MAX) and the
    factor-iterations all ranks processed (SUM)."""
    el = torch.tensor([elapsed], device=device, dtype=torch.float64)
    fi = torch.tensor([float(factor_iters)], device=device, dtype=torch.float64)
    if world > 1 or USE_DIST:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        dist.all_reduce(fi, op=dist.ReduceOp.SUM)
    return float(el.item()), float(fi.item())


PEAK_F16_MFMA = 16 * PEAK_F32  # TFLOP/s dense f16 MFMA (MI355X_MICROARCH.md: 1/16 rate ratio, ~2.5 PF)
PEAK_HBM = 8.0                 # TB/s HBM3E spec
THIN_ROWS = 16                 # kThinRows: factors with I <= 16 take k_thin_solve / k_mse_small_admm or k_thin_loop
SPLIT_PRODUCTS = 3             # split-fp16 solve: Ph Mh + Ph Ml + Pl Mh per solve flop

# Launch classes of admmq_profile_end (include/admmq.h ADMMQ_PROF_*) and, per element of
# an (I, R) factor (or per factor), the algorithmic work one launch does for one
# problem. Bytes are the compulsory HBM bytes of DESIGN.md §4 (fp32 = 4 B; the split
# planes are 2 x 2 B = 4 B per element too):
#   gemm / gemm_thin  H_T = P M: 2 I R^2 flops; read P, U, M, write H_T: 4 (3 I R + R^2) B
#   search            stage 1 + selection + stage 2 over X = H_T - U: read H_T, U: 8 I R B;
#                     with the finalize fused into the launch (k_mse_hist3<.., true>): 28 I R B
#                     (SURVEY §8(d) counts the reference's exhaustive sweep, 8 x 200 flops
#                     per element; reported beside the byte roofline as `valu_equiv`)
#   small             search + finalize of the I <= 16 factors in one block: 8 I R + 28 I R B
#   finalize          read H_T, H, U, F, write H, U, next P: 28 I R B
#   thin_loop         every iteration of an all-thin call in one launch (k_thin_loop):
#                     (max_iter - 1) x 2 I R^2 solve flops; compulsory HBM bytes once per
#                     call: M, F, H, U, P in, H, U out: 4 (R^2 + 6 I R) B
PROF_CLASSES = ["gemm", "gemm_thin", "search", "small", "finalize", "prepare", "thin_loop"]
PER_ITER_CLASSES = PROF_CLASSES[:5]
KERNEL_NAMES = {"gemm": "k_gemm (solve GEMM)", "gemm_thin": "k_thin_solve (solve, I<=16, VALU)",
                "search": "k_mse_hist3 (two-stage MSE search)", "small": "k_mse_small_admm (I<=16 search+finalize)",
                "finalize": "k_finalize_admm (projection + dual update)", "prepare": "prepare (rho, SPD inverse, planes)",
                "thin_loop": "k_thin_loop (persistent: every iteration of the I<=16 factors, VALU solve)"}


def mode_problems(work):
    """[(I, R) of every factor solved in mode m] per mode m (bench batches one mode of
    every layer per admm_iteration_batched call, like admmq.factorize.als_sweep)."""
    nm = max(len(s.shape) for (s, _, _, _) in work)
    return [[(s.shape[m], R) for (s, _, R, _) in work if m < len(s.shape)] for m in range(nm)]


def class_work(work, num_attempts=200, split=True, fused=False, max_iter_admm=1000):
    """Per launch class: (flops, bytes, valu_equiv_flops) of ONE launch, averaged over the
    modes whose calls issue it. The HIP-event sampling times one iteration in N of every
    mode call, so each issuing mode weighs equally in the measured average duration."""
    out = {}
    loop = [[(i, r) for (i, r) in probs] for probs in mode_problems(work) if all(i <= THIN_ROWS for (i, _) in probs)]
    if loop:
        n = len(loop)
        out["thin_loop"] = (sum((max_iter_admm - 1) * 2.0 * i * r * r for p in loop for (i, r) in p) / n,
                            sum(4.0 * (r * r + 6 * i * r) for p in loop for (i, r) in p) / n,
                            sum((max_iter_admm - 1) * 8.0 * num_attempts * i * r for p in loop for (i, r) in p) / n)
    for cls in PER_ITER_CLASSES:
        per_mode = []
        for probs in mode_problems(work):
            big = [(i, r) for (i, r) in probs if i > THIN_ROWS]
            thin = [(i, r) for (i, r) in probs if i <= THIN_ROWS]
            sel = thin if cls in ("gemm_thin", "small") else big
            if not sel:
                continue
            fl = sum(2.0 * i * r * r for (i, r) in sel) if cls.startswith("gemm") else 0.0
            if cls.startswith("gemm"):
                by = sum(4.0 * (3 * i * r + r * r) for (i, r) in sel)
            elif cls == "search":   # fused: + the finalize step's H, F reads and H, U, P writes
                by = sum((28.0 if fused else 8.0) * i * r for (i, r) in sel)
            elif cls == "small":
                by = sum(36.0 * i * r for (i, r) in sel)
            else:
                by = sum(28.0 * i * r for (i, r) in sel)
            ve = sum(8.0 * num_attempts * i * r for (i, r) in sel) if cls in ("search", "small") else 0.0
            per_mode.append((fl, by, ve))
        if per_mode:
            n = len(per_mode)
            out[cls] = tuple(sum(x[k] for x in per_mode) / n for k in range(3))
    return out


def kernel_roofline(cls, work_tuple, avg_us, launches, split, traffic):
    """Roofline of one launch class: bound = the larger of its MFMA and HBM times at peak
    (solve: f16 MFMA / 3 products when split, fp32 MFMA otherwise); achieved = algorithmic
    work per launch / measured average launch duration."""
    fl, by, ve = work_tuple
    t = avg_us * 1e-6
    mf_peak = (PEAK_F16_MFMA / SPLIT_PRODUCTS) if (split and cls == "gemm") else PEAK_F32
    t_mfma = fl / (mf_peak * 1e12) if fl else 0.0
    t_hbm = by / (PEAK_HBM * 1e12)
    if t_mfma > t_hbm:
        r = {"bound": "mfma", "achieved": fl / t / 1e12, "peak": mf_peak, "unit": "TFLOP/s"}
    else:
        r = {"bound": "hbm", "achieved": by / t / 1e9, "peak": PEAK_HBM * 1e3, "unit": "GB/s"}
    r["frac"] = r["achieved"] / r["peak"]
    tr = (traffic or {}).get("classes", {}).get(cls)
    r["traffic"] = tr["bytes_per_launch"] if tr else None
    r.update({"traffic_unit": "HBM bytes/launch (PMC: 2 FETCH_SIZE + WRITE_SIZE)", "kernel": KERNEL_NAMES[cls],
              "launch_avg_us": avg_us, "launches_timed": launches, "algorithmic_bytes_per_launch": by,
              "algorithmic_flops_per_launch": fl, "t_ideal_us": max(t_mfma, t_hbm) * 1e6})
    if cls == "gemm":
        r["kernel"] = ("k_gemm (solve, split-f16 MFMA)" if split
                       else "k_gemm_f32b (solve, fp32 MFMA; 256x128 k_gemm tiles in many-round launches)")
        r["mfma_form"] = "split-f16 (v_mfma_f32_32x32x16_f16, 3 products)" if split else "fp32 (v_mfma_f32_32x32x2_f32)"
    if ve:
        r["valu_equiv"] = {"achieved": ve / t / 1e12, "peak": PEAK_F32, "unit": "TFLOP/s",
                           "frac": ve / t / 1e12 / PEAK_F32,
                           "note": "SURVEY §8(d) F_valu: the reference's 200-candidate sweep, 8 flops/candidate-element"}
    if traffic:
        r["traffic_source"] = traffic["file"]
    return r


def step_roofline(work, max_iter_admm, ms_per_step, num_attempts=200):
    """T_ideal = max(F_mfma / 157.3 TF/s, F_valu / 157.3 TF/s, B_hbm / 8 TB/s)
    per factor-iteration, summed over every (layer, mode) x inner iteration of the step."""
    it = max_iter_admm - 1
    f_mfma = sum(2.0 * I * R * R for probs in mode_problems(work) for (I, R) in probs) * it
    f_valu = sum((8.0 * num_attempts + 20.0) * I * R for probs in mode_problems(work) for (I, R) in probs) * it
    b_hbm = sum(4.0 * (6 * I * R + R * R) for probs in mode_problems(work) for (I, R) in probs) * it
    terms = {"mfma_fp32": f_mfma / (PEAK_F32 * 1e12), "valu": f_valu / (PEAK_F32 * 1e12), "hbm": b_hbm / (PEAK_HBM * 1e12)}
    t_ideal = max(terms.values())
    # the same step with the solve priced at the form it runs in (split: f16 MFMA, 3
    # products); the §8(d) figure above prices it at the fp32 MFMA peak, which the split
    # solve can beat (frac > 1 at C5)
    t_split = max(f_mfma / (PEAK_F16_MFMA / SPLIT_PRODUCTS * 1e12), terms["valu"], terms["hbm"])
    return {"t_ideal_ms": t_ideal * 1e3, "t_measured_ms": ms_per_step, "frac": t_ideal * 1e3 / ms_per_step,
            "terms_ms": {k: v * 1e3 for k, v in terms.items()}, "binding": max(terms, key=terms.get),
            "formula": "SURVEY §8(d): max(F_mfma/157.3 TF/s, F_valu/157.3 TF/s, B_hbm/8 TB/s) per step",
            "t_ideal_split_solve_ms": t_split * 1e3, "frac_split_solve": t_split * 1e3 / ms_per_step,
            "split_solve_note": "solve term at the split form's f16 MFMA peak / 3 products (838.9 TF/s)"}


TRAFFIC_TAGS = ("r06", "r05", "r04", "r03")   # newest first


def load_traffic(model, split):
    """Per-launch HBM bytes of each launch class from the committed rocprofv3 PMC passes of
    THIS config (profiles/<tag>_<model>_traffic.json, tools/traffic_json.py; the newest
    round that profiled it); PMC counters cannot be read live inside the timed region. None
    when no file matches the config."""
    t = None
    for tag in TRAFFIC_TAGS:
        path = os.path.join(ROOT, "profiles", f"{tag}_{model}_traffic.json")
        try:
            with open(path) as f:
                cand = json.load(f)
        except (OSError, ValueError):
            continue
        if cand.get("split", True) == split:
            t = cand
            break
    if t is None:
        return None
    t["file"] = os.path.relpath(path, ROOT)
    return t


def cpu_baseline(work, max_iter_admm, sample_iters=20):
    """torch-CPU port of the reference step (oracle/torch_port.py) on a bounded sample:
    every DISTINCT (layer shape, rank, mode) problem of the workload runs its setup plus
    `sample_iters` inner iterations on the host cores; the per-iteration cost (constant
    with eps=0) is extrapolated to max_iter_admm-1 iterations and weighted by how many
    (layer, mode) problems of the workload share that shape."""
    from oracle import torch_port
    classes = {}
    for (s, W, R, init) in work:
        for m in range(len(s.shape)):
            key = (tuple(s.shape), R, m)
            if key not in classes:
                classes[key] = [0, W, init]
            classes[key][0] += 1
    total = 0.0
    n_fi = 0
    wall = time.time()
    for (shape, R, m), (count, W, init) in classes.items():
        Wc = W.cpu()
        fs = [f.cpu() for f in init]
        G, F = torch_port.gram_mttkrp(Wc, fs, m)
        t0 = time.perf_counter()
        torch_port.admm_iteration(fs[m], torch.zeros_like(fs[m]), F, G, 1, 0.0, 4)
        t1 = time.perf_counter()
        torch_port.admm_iteration(fs[m], torch.zeros_like(fs[m]), F, G, 1 + sample_iters, 0.0, 4)
        t2 = time.perf_counter()
        setup = t1 - t0
        per_iter = max((t2 - t1) - setup, 0.0) / sample_iters
        total += count * (setup + per_iter * (max_iter_admm - 1))
        n_fi += count * (max_iter_admm - 1)
    nprob = sum(c[0] for c in classes.values())
    return {"value": n_fi / total, "unit": "factor-iterations/s", "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"{len(classes)} distinct (shape, rank, mode) problems of the workload's {nprob}: setup + "
                      f"{sample_iters} inner iterations each timed on host cores (torch-CPU port of source/admm.py + "
                      f"quantization.py, oracle/torch_port.py), extrapolated to {max_iter_admm - 1} iterations and "
                      f"weighted by multiplicity; {time.time() - wall:.1f}s of CPU work"}


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


def time_steps(work, max_iter_admm, steps, warmup):
    for _ in range(warmup):
        run_step(work, max_iter_admm)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        run_step(work, max_iter_admm)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / steps


def class_avgs(work, max_iter_admm, every=8):
    """One profiled sweep: average microseconds per launch of each kernel class (HIP events
    on the library's stream, every `every`-th iteration)."""
    import ctypes
    from admmq import _lib
    lib = _lib.load()
    _lib.check(lib.admmq_profile_begin(3 * 6 * (max_iter_admm // every + 1) + 64, every), "profile_begin")
    run_step(work, max_iter_admm)
    torch.cuda.synchronize()
    ms = (ctypes.c_double * 8)()
    cnt = (ctypes.c_int64 * 8)()
    _lib.check(lib.admmq_profile_end(ms, cnt), "profile_end")
    return {c: round(1e3 * ms[i] / cnt[i], 2) for i, c in enumerate(PROF_CLASSES) if cnt[i]}


def emulate_shards(a):
    """SURVEY §8(e) readiness without a node: every rank's LPT shard of an N-GPU
    `--shard layers` run (bench.build_workload with that rank / world) is timed on this
    one GPU with the same code path, plus the whole model; the implied N-GPU strong-scaling
    speed-up is the whole model's ms per sweep over the busiest shard's (the final gather
    of factors, ~20-400 MB over xGMI, is not included)."""
    torch.cuda.set_device(0)
    device = torch.device("cuda", 0)
    from admmq import _lib
    lib = _lib.load()
    _lib.check(lib.admmq_set_solve_mode(0 if a.solve == "fp32" else 1), "set_solve_mode")
    _lib.check(lib.admmq_debug_set_ksplit(a.ksplit), "ksplit")
    _lib.check(lib.admmq_debug_set_ksplit_form(a.ksplit_form), "ksplit_form")
    _lib.check(lib.admmq_debug_set_ksplit_balance(*[int(v) for v in a.ksplit_bal.split(":")]), "ksplit_balance")
    _lib.check(lib.admmq_debug_set_fin_nv3(a.fin_nv3), "fin_nv3")
    if a.gemm_stage >= 0:
        _lib.check(lib.admmq_debug_set_gemm_stage(a.gemm_stage), "gemm_stage")
    N = a.emulate_world
    only = [int(v) for v in a.emulate_only.split(",")] if a.emulate_only else None
    full_ms = None
    if only is None:
        full, _, _ = build_workload(a.model, 0, 1, "layers", device)
        full_ms = time_steps(full, a.max_iter_admm, a.steps, a.warmup)
        del full
    shard_ms, nlayers, info, shard_us, shard_cost = [], [], None, [], []
    for r in (only if only is not None else range(N)):
        work, _, info = build_workload(a.model, r, N, "layers", device)
        shard_cost.append(sum(layer_cost(s, R) for (s, _, R, _) in work))
        nlayers.append(len(work))
        shard_ms.append(time_steps(work, a.max_iter_admm, a.steps, a.warmup) if work else 0.0)
        shard_us.append(class_avgs(work, a.max_iter_admm) if work else {})
        del work
        print(f"shard {r}/{N}: {nlayers[-1]} layers, {shard_ms[-1]:.1f} ms per sweep", file=sys.stderr, flush=True)
    out = {"metric": "emulated layer-shard sweep time (one GPU)", "model": a.model, "world": N, "solve": a.solve,
           "max_iter_admm": a.max_iter_admm, "steps": a.steps, "full_ms_per_sweep": full_ms,
           "shard_ms_per_sweep": shard_ms, "layers_per_rank": nlayers, "busiest_ms": max(shard_ms),
           "shard_cost": shard_cost, "total_cost": sum(layer_cost(s, s.rank()) for s in _model_specs(a.model)),
           "shard_kernel_avg_us": shard_us,
           "ranks": only if only is not None else list(range(N)),
           "implied_speedup": full_ms / max(shard_ms) if full_ms else None, "lpt_speedup_cap": info["lpt_speedup_cap"],
           "whole_layer_speedup_cap": info["whole_layer_speedup_cap"], "policy": info["policy"]}
    print(json.dumps(out), flush=True)


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n):
    """`python bench.py --gpus N` (no WORLD_SIZE): run the same command under
    torch.distributed.run with N ranks on this node (rendezvous on 127.0.0.1) as a CHILD
    process - this parent never initialises the GPU, so no exec from a GPU process - relay
    its output and exit with its code. Rank 0 prints the JSON line."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    sys.exit(subprocess.call(cmd, env=env))


def dry_run(a, world, rank):
    """--cpu-dry-run: the multi-rank plumbing of a real run on CPU tensors over gloo - the
    LPT shard plan, warmup + K timed (kernel-free) steps between barriers, the single factor
    gather to rank 0 and the max / sum reductions - so a CPU test can check that `--gpus N`
    forms N ranks and that rank 0 receives every layer's factors."""
    device = torch.device("cpu")
    if USE_DIST:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    work, numel, shard_info = build_workload(a.model, rank, world, a.shard, device)
    got, keep = 0, []
    t0 = time.perf_counter()
    for _ in range(a.warmup + a.steps):
        runs = [type("Run", (), {"factors": [f.clone() for f in init]})() for (_, _, _, init) in work]
        got = gather_factors(runs, rank, world, numel, device, keep)
    if USE_DIST:
        dist.barrier()
    elapsed, nfi = reduce_over_ranks(time.perf_counter() - t0, len(work), world, device)
    if rank == 0:
        # every rank's gathered buffer equals that rank's own factors (here: its seeded init)
        match = []
        for k in range(world):
            wk, _, _ = build_workload(a.model, k, world, a.shard, device)
            ref = torch.cat([f.reshape(-1) for (_, _, _, init) in wk for f in init]) if wk else torch.zeros(0)
            match.append(bool(torch.equal(keep[k], ref)))
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_formed": world, "gathered_elements": got,
                          "expected_elements": sum(numel), "layers_total": int(nfi),
                          "layers_per_rank": (shard_info or {}).get("layers_per_rank"),
                          "rank_factors_match": match, "elapsed_s": elapsed}), flush=True)
    if USE_DIST:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--max-iter-admm", type=int, default=1000)
    ap.add_argument("--shard", choices=["layers", "replica"], default="layers",
                    help="layers: LPT-shard one model's layers over the ranks (default); replica: every rank its own copy")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-iters", type=int, default=None,
                    help="inner iterations timed per (layer, mode) on the CPU (default 20; 1 for llama7b)")
    ap.add_argument("--no-profile", action="store_true", help="skip the live HIP-event kernel timing")
    ap.add_argument("--prof-every", type=int, default=16,
                    help="HIP-event timing of one ADMM iteration in N (GEMM and search: events recorded by the "
                         "dispatch itself, the kernel's own time; the other classes: an event pair per launch)")
    ap.add_argument("--solve", choices=["split", "fp32"], default="fp32",
                    help="per-iteration solve GEMM form: fp32 MFMA (default: the reference's fp32 arithmetic) or "
                         "split-fp16 planes on f16 MFMA (opt-in, ~22-bit operands; never the headline)")
    ap.add_argument("--exhaustive", action="store_true",
                    help="A/B: evaluate all MSE candidates (reference-style) instead of the two-stage search")
    ap.add_argument("--search-units", type=int, default=0,
                    help="A/B: stage-1 units per block of the non-fused search launch (0: the planner's choice)")
    ap.add_argument("--f32-kernel", type=int, default=-1,
                    help="A/B: fp32 solve kernel 0 = k_gemm, 1 = persistent lists, 2 = one tile per workgroup with "
                         "per-problem tile rows (-1: library default)")
    ap.add_argument("--f32-tiles", type=int, default=3, help="A/B: tile-row rule 0..3 of --f32-kernel 1 / 2")
    ap.add_argument("--gemm-ks", type=int, default=1, help="A/B: fp32 64x64 tiles with 4 (1) or 8 (2) waves")
    ap.add_argument("--ksplit", type=int, default=1, choices=[0, 1],
                    help="A/B: K-split of the fp32 solve tiles of factors too small to fill the chip (1, default: "
                         "pieces fixed by each factor's shape) or never (0)")
    ap.add_argument("--wide-min", type=int, default=-1,
                    help="diagnostics: 64x64 tiles per launch from which factors take 256x128 tiles (default 3072)")
    ap.add_argument("--emulate-only", default="",
                    help="with --emulate-world: time only these ranks' shards (comma list), not the whole model")
    ap.add_argument("--ksplit-form", type=int, default=1, choices=[0, 1, 2],
                    help="A/B: K-split pieces run in parallel where the launch leaves CUs idle (1, default), always "
                         "serially in one workgroup (0) or always in parallel (2); same bits")
    ap.add_argument("--ksplit-bal", default="1:1",
                    help="A/B: ON:COST - run the pieces of the longest split tiles in parallel where that lowers "
                         "the launch's CU-level LPT makespan (a parallel piece priced COST K-steps extra); same bits")
    ap.add_argument("--gemm-stage", type=int, default=-1,
                    help="A/B: fp32 64x64 staging form 0..4 (library default 3; 2 = 2-deep ring, 4 tiles per CU)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise torch.distributed (RCCL) and run the gather / all-reduce even at N = 1 "
                         "(launch under torch.distributed.run): exercises the multi-GPU path on one GPU")
    ap.add_argument("--fin-nv3", type=int, default=1, choices=[0, 1],
                    help="A/B: 1 (library default) = three float4 groups per search thread where that keeps the "
                         "finalize in the search launch (C4), 0 = at most two (separate finalize launch at C4)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="multi-GPU readiness on ONE GPU: time every rank's LPT layer shard of an N-GPU run "
                         "(same code path, one after another) and report the busiest shard and the implied speed-up")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="tests only: no GPU, no kernels - the launcher, the shard plan and the factor gather over "
                         "gloo on CPU tensors (the factors are the init, unchanged)")
    a = ap.parse_args()
    if a.emulate_world > 0:
        return emulate_shards(a)

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        # --gpus N without a launcher: start N rank processes as children (torch.distributed.run);
        # this process never touches the GPU (no exec from a GPU-initialised process)
        return launch_ranks(a.gpus)
    world = int(env_world or "1")
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher formed WORLD_SIZE={world}; refusing to report a "
              f"{world}-rank run as {a.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    global USE_DIST
    USE_DIST = world > 1 or a.force_dist
    if a.cpu_dry_run:
        return dry_run(a, world, rank)
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if USE_DIST:
        dist.init_process_group("nccl", device_id=device)
        world = dist.get_world_size()   # n_gpus from the world actually formed

    from admmq import _lib
    lib = _lib.load()
    lib.admmq_set_exhaustive_search(1 if a.exhaustive else 0)
    _lib.check(lib.admmq_set_solve_mode(0 if a.solve == "fp32" else 1), "set_solve_mode")
    _lib.check(lib.admmq_debug_set_search_units_per_block(a.search_units), "search_units_per_block")
    _lib.check(lib.admmq_debug_set_gemm_ks(a.gemm_ks), "gemm_ks")
    _lib.check(lib.admmq_debug_set_ksplit(a.ksplit), "ksplit")
    _lib.check(lib.admmq_debug_set_ksplit_form(a.ksplit_form), "ksplit_form")
    _lib.check(lib.admmq_debug_set_ksplit_balance(*[int(v) for v in a.ksplit_bal.split(":")]), "ksplit_balance")
    if a.gemm_stage >= 0:
        _lib.check(lib.admmq_debug_set_gemm_stage(a.gemm_stage), "gemm_stage")
    if a.wide_min >= 0:
        _lib.check(lib.admmq_debug_set_wide_min_tiles(a.wide_min), "wide_min")
    _lib.check(lib.admmq_debug_set_fin_nv3(a.fin_nv3), "fin_nv3")
    if a.f32_kernel >= 0:
        _lib.check(lib.admmq_debug_set_f32_persistent(a.f32_kernel, a.f32_tiles), "f32_kernel")
    split = a.solve == "split"
    work, numel, shard_info = build_workload(a.model, rank, world, a.shard, device)
    fi_per_step = sum(len(s.shape) * (a.max_iter_admm - 1) for (s, _, _, _) in work)

    for _ in range(a.warmup):
        gather_factors(run_step(work, a.max_iter_admm), rank, world, numel, device)
    torch.cuda.synchronize()

    _lib.fault_repairs(reset=True)   # fused-path faults repaired by a re-run inside the timed steps (expected 0)
    prof = not a.no_profile
    if prof:
        n_launch = a.steps * 3 * 6 * (a.max_iter_admm // a.prof_every + 1) + 64
        _lib.check(lib.admmq_profile_begin(n_launch, a.prof_every), "profile_begin")
    if USE_DIST:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        runs = run_step(work, a.max_iter_admm)
        gather_factors(runs, rank, world, numel, device)
    torch.cuda.synchronize()
    if USE_DIST:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern = None
    if prof:
        import ctypes
        ms = (ctypes.c_double * 8)()
        cnt = (ctypes.c_int64 * 8)()
        _lib.check(lib.admmq_profile_end(ms, cnt), "profile_end")
        kern = {"ms": list(ms), "launches": list(cnt)}

    repairs = _lib.fault_repairs()
    elapsed_max, total_fi = reduce_over_ranks(elapsed, fi_per_step * a.steps, world, device)

    if rank == 0:
        out = {"metric": METRIC, "value": total_fi / elapsed_max, "unit": "factor-iterations/s", "n_gpus": world,
               "steps": a.steps, "warmup": a.warmup, "ms_per_step": 1e3 * elapsed_max / a.steps,
               "higher_is_better": True, "scaling": "weak" if a.shard == "replica" else "strong",
               "vs_baseline": None,
               "dtype": "f32 (solve: split-f16 MFMA, fp32 accumulate)" if split else "f32", "data": "synthetic",
               "config": {"workload": workload_name(a.model, work, a.max_iter_admm),
                          "factor_iterations_per_step_per_gpu": fi_per_step, "max_iter_admm": a.max_iter_admm,
                          "parallelism": f"{'replica' if a.shard == 'replica' else 'layer-shard'} x{world}, "
                                         "one RCCL gather of factors per step",
                          "mse_search": "exhaustive" if a.exhaustive else "two-stage exact",
                          "solve": a.solve}}
        out["step_roofline"] = step_roofline(work, a.max_iter_admm, out["ms_per_step"])
        out["finalize_repairs"] = repairs   # rank 0's calls re-run after a fused-path internal fault
        if shard_info:
            out["config"]["shard"] = shard_info
        if kern is not None:
            ms, cnt = kern["ms"], kern["launches"]
            avg_us = {c: 1e3 * ms[i] / cnt[i] for i, c in enumerate(PROF_CLASSES) if cnt[i]}
            traffic = load_traffic(a.model, split)
            fused = "search" in avg_us and "finalize" not in avg_us   # the big jobs' finalize ran in the search launch
            cw = class_work(work, split=split, fused=fused, max_iter_admm=a.max_iter_admm)
            rf = {c: kernel_roofline(c, cw[c], avg_us[c], cnt[i], split, traffic)
                  for i, c in enumerate(PROF_CLASSES) if c in cw and c in avg_us}
            if fused and "search" in rf:
                rf["search"]["kernel"] = "k_mse_hist3 (two-stage MSE search + fused finalize)"
            # per step: each class launches once per inner iteration of every mode that issues it
            # (all-thin calls run as one k_thin_loop launch instead: per call, every call timed)
            per_iter_modes = [p for p in mode_problems(work) if not (cnt[PROF_CLASSES.index("thin_loop")] and
                                                                     all(i <= THIN_ROWS for (i, _) in p))]
            n_issuing = {c: sum(1 for probs in per_iter_modes
                                if any((i <= THIN_ROWS) == (c in ("gemm_thin", "small")) for (i, _) in probs))
                         for c in PER_ITER_CLASSES}
            per_step = {c: avg_us[c] * 1e-3 * n_issuing[c] * (a.max_iter_admm - 1) for c in rf if c in n_issuing}
            for c in ("prepare", "thin_loop"):
                if c in avg_us:
                    per_step[c] = avg_us[c] * 1e-3 * cnt[PROF_CLASSES.index(c)] / a.steps
            dom = max(rf, key=lambda c: per_step[c])
            out["roofline"] = rf[dom]
            out["roofline_kernels"] = rf
            out["kernel_ms_per_step"] = per_step
            out["kernel_avg_us"] = avg_us
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
    if USE_DIST:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

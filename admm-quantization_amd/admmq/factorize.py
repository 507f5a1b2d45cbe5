"""ALS driver of the ADMM quantized CP factorization (``scripts/factorize.py``).

``factorize_layers`` runs the reference's per-layer loop (3-way
``scripts/factorize.py:207-266``, 2-way ``:269-310``) for MANY independent layers at
once: in each ALS sweep, mode m of every active layer is solved in one batched
``admm_iteration_batched`` launch sequence, followed by one batched re-quantization.
Per layer it keeps the reference's semantics exactly: modes in order A -> B -> C
with each mode using the factors already updated in this sweep, duals carried
across sweeps, the two reconstruction errors per sweep and the stop tests
(|dloss| < tol, exploding error over 5 (3-way) or 10 (2-way) sweeps).

``main()`` mirrors the reference CLI (same flag names) and output files
(``{bits}bit_{qscheme}/factors_{method}_seed{seed}/{layer}_{method}_{init}_rank_{R}_mode_{n}.pt``
plus ``_losshist.pt`` / ``_lossquanthist.pt``). Pretrained weights cannot be
downloaded here, so weights come from ``--weights`` (a state_dict loaded with
``weights_only=True``) or from the seeded synthetic generator of
:mod:`admmq.synthetic`. The reference's own script crashes before reaching this
loop; the intended 4-D -> 3-D reshape of ``:140-147`` is applied.
"""
from __future__ import annotations

import argparse
import json
import os
import time
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from . import _lib, synthetic
from .admm import admm_iteration_batched, init_factors_many
from .als import gram_mttkrp, gram_mttkrp_batched, rel_error_batched  # noqa: F401
from .quantization import quantize_batched


def reconstruct(factors: Sequence[torch.Tensor]) -> torch.Tensor:
    """[[factors]] as a dense tensor (torch; for callers that need the tensor itself -
    the ALS driver's errors use the fused ``als.rel_error_batched`` instead)."""
    if len(factors) == 3:
        return torch.einsum('ir,jr,kr->ijk', *factors)
    return factors[0] @ factors[1].T


@dataclass
class LayerRun:
    name: str
    W: torch.Tensor
    rank: int
    factors: List[torch.Tensor]
    duals: List[torch.Tensor] = field(default_factory=list)
    quantized: List[Optional[torch.Tensor]] = field(default_factory=list)
    loss: List[float] = field(default_factory=list)
    lossq: List[float] = field(default_factory=list)
    active: bool = True
    # What the reference saves (scripts/factorize.py:315-318): the 3-way loop assigns
    # `factors` after the loop (the latest sweep); the 2-way loop assigns it at the
    # end of each sweep body, after the stop tests (:309-310), so a break leaves the
    # previous sweep's factors (the initial ones before the first full sweep).
    saved: List[torch.Tensor] = field(default_factory=list)
    saved_quantized: List[Optional[torch.Tensor]] = field(default_factory=list)

    def __post_init__(self):
        if not self.duals:
            self.duals = [torch.zeros_like(f) for f in self.factors]
        if not self.quantized:
            self.quantized = [None] * len(self.factors)
        if not self.saved:
            self.saved = list(self.factors)
            self.saved_quantized = list(self.quantized)

    def result(self):
        """(factors, quantized factors) as the reference's script would save them."""
        if self.W.dim() == 3:
            return list(self.factors), list(self.quantized)
        return list(self.saved), list(self.saved_quantized)


def als_sweep(runs: Sequence[LayerRun], max_iter_admm: int, eps: float, bits: int, qscheme: str,
              num_attempts: int = 200, record_errors: bool = True, tol: float = 1e-5, solve: Optional[str] = None):
    """One ALS sweep over all active layers (modes batched across layers). Returns the
    factor-iterations the inner ADMM loops ran in this sweep, per active layer
    (``{id(run): count}``).

    SPD failures and internal faults are read once per sweep (one host sync):
    * a ``LinAlgError`` is raised after every mode of the sweep has run, so - unlike the
      reference, which raises at the Cholesky call before changing anything
      (``source/admm.py:54``) - the runs' factors, duals and quantized factors are
      undefined after the error;
    * an internal fault of a fused path (its bounded wait expired: another stream's work
      broke its residency assumption, include/admmq.h) restores the sweep's starting
      factors, duals and quantized factors and re-runs the whole sweep without the fused
      paths (later modes read the earlier modes' results, so a faulted call cannot be
      repeated alone); the repair is counted in ``_lib.fault_repairs``."""
    act = [r for r in runs if r.active]
    nmodes = max((len(r.factors) for r in act), default=0)
    # the sweep's starting point (factors and quantized factors are rebound, duals updated in place)
    start = [(list(r.factors), [u.clone() for u in r.duals], list(r.quantized)) for r in act]

    def modes(check_fault):
        infos = []
        for mode in range(nmodes):
            sel = [r for r in act if mode < len(r.factors)]
            GF = gram_mttkrp_batched([(r.W, r.factors) for r in sel], mode)
            probs = [(r.factors[mode], r.duals[mode], F, G) for r, (G, F) in zip(sel, GF)]
            # no per-call sync for the SPD and fault tests: the flags are read once per sweep (below)
            Hs, info = admm_iteration_batched(probs, max_iter_admm, eps, bits, qscheme, num_attempts=num_attempts,
                                              check_spd=False, return_info=True, solve=solve, check_fault=check_fault)
            infos.append(info[:, [0, 2, 3]])   # {iterations run, spd_error, internal fault}
            for r, H in zip(sel, Hs):
                r.factors[mode] = H
            qs = quantize_batched(Hs, bits, qscheme, num_attempts=num_attempts)
            for r, q in zip(sel, qs):
                r.quantized[mode] = q
        return torch.cat(infos).cpu() if infos else None   # the sweep's one host sync for the flags

    both = modes(False)
    if both is not None and int(both[:, 2].max()) != 0:   # internal fault: the sweep again, without the fused paths
        for r, (fs, us, qs) in zip(act, start):
            r.factors[:] = fs
            for u, u0 in zip(r.duals, us):
                u.copy_(u0)
            r.quantized[:] = qs
        with _lib.fused_finalize(False):
            both = modes(True)
        _lib.note_repair()
    iters = {id(r): 0 for r in act}
    if both is not None:
        check_spd_flags([both[:, 1]], act, nmodes)
        k = 0
        for mode in range(nmodes):
            for r in (r for r in act if mode < len(r.factors)):
                iters[id(r)] += int(both[k, 0])
                k += 1
    if not record_errors:
        return iters
    errs = rel_error_batched([(r.W, r.factors) for r in act] + [(r.W, r.quantized) for r in act])
    for n, r in enumerate(act):
        r.loss.append(errs[n])
        r.lossq.append(errs[len(act) + n])
        back = 5 if r.W.dim() == 3 else 10
        if len(r.loss) > 1 and abs(r.loss[-2] - r.loss[-1]) < tol:
            r.active = False
        elif len(r.loss) > 10 and r.loss[-1] - r.loss[-back] > 1e-3:
            r.active = False
        else:   # the 2-way script's end-of-body assignment (scripts/factorize.py:309-310)
            r.saved, r.saved_quantized = list(r.factors), list(r.quantized)
    return iters


def check_spd_flags(infos, runs, nmodes):
    """source/admm.py:54 raises torch.linalg.LinAlgError when G + rho I is not SPD.
    The batched driver reads every mode's device flag in ONE host sync per sweep and
    raises the same error, naming the first failing (layer, mode)."""
    flags = torch.cat(infos).cpu()
    if int(flags.max()) == 0:
        return
    k = int(torch.nonzero(flags)[0])
    for mode in range(nmodes):
        sel = [r for r in runs if mode < len(r.factors)]
        if k < len(sel):
            raise torch.linalg.LinAlgError(f"linalg.cholesky: The factorization could not be completed because the "
                                           f"input is not positive-definite (layer {sel[k].name}, mode {mode}).")
        k -= len(sel)


def factorize_layers(weights: Sequence[torch.Tensor], ranks: Sequence[int], max_iter_als: int, max_iter_admm: int,
                     bits: int = 4, qscheme: str = "tensor_mseminmax_symmetric", init: str = "random", seed: int = 42,
                     names: Optional[Sequence[str]] = None, eps: float = 1e-8, tol: float = 1e-5,
                     num_attempts: int = 200, initial_factors=None, metrics=None) -> List[LayerRun]:
    """``--method admm`` of scripts/factorize.py for a batch of layers.

    ``metrics``: optional callable receiving one dict per (sweep, layer) - the keys the
    reference logs to wandb per ALS iteration (``rec_error``, ``quant_rec_error``,
    scripts/factorize.py:249-253, 301-305) plus the sweep's wall time and ADMM
    factor-iterations (see :func:`sweep_records`)."""
    runs = []
    if initial_factors is None:   # every layer's init at once (parafac-epc: one stream per layer)
        initial_factors = init_factors_many(weights, ranks, init=init, device=weights[0].device if weights else None,
                                            seed=seed)
    for i, (W, R) in enumerate(zip(weights, ranks)):
        fs = [f.to(W.device).contiguous().clone() for f in initial_factors[i]]
        run = LayerRun(names[i] if names else f"layer{i}", W, R, fs)
        if init != "random":   # scripts/factorize.py:192-204: record the starting point
            q = quantize_batched(fs, bits, qscheme, num_attempts=num_attempts)
            e, eq = rel_error_batched([(W, fs), (W, q)])
            run.loss.append(e)
            run.lossq.append(eq)
            run.saved_quantized = list(q)
        runs.append(run)
    for sweep in range(max_iter_als):
        if not any(r.active for r in runs):
            break
        act = [r for r in runs if r.active]
        t0 = time.perf_counter()
        iters = als_sweep(runs, max_iter_admm, eps, bits, qscheme, num_attempts=num_attempts, tol=tol)
        dt = time.perf_counter() - t0   # the errors above were read on the host: the sweep is complete
        if metrics is not None:
            for rec in sweep_records(act, sweep, iters, dt):
                metrics(rec)
    return runs


def sweep_records(runs: Sequence[LayerRun], sweep: int, iters: dict, seconds: float) -> List[dict]:
    """JSONL metric records of one ALS sweep (the reference prints / logs
    to wandb; this build writes one JSON object per (sweep, layer)). ``sweep_s`` and
    ``factor_iterations_per_s`` are for the whole batched sweep (all layers share its
    launches); ``factor_iterations`` is the layer's own inner-iteration count."""
    total = sum(iters.values())
    out = []
    for r in runs:
        out.append({"sweep": sweep, "layer": r.name, "rank": r.rank,
                    "rec_error": r.loss[-1] if r.loss else None,
                    "quant_rec_error": r.lossq[-1] if r.lossq else None,
                    "factor_iterations": int(iters.get(id(r), 0)), "active": bool(r.active),
                    "sweep_s": seconds, "factor_iterations_per_s": (total / seconds) if seconds > 0 else None})
    return out


class JsonlWriter:
    """Appends one JSON object per line to ``path`` (flushed per record)."""

    def __init__(self, path: str):
        self.path = path
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        self._f = open(path, "a")

    def __call__(self, rec: dict):
        self._f.write(json.dumps(rec) + "\n")
        self._f.flush()

    def close(self):
        self._f.close()


def _layer_weight(args, device):
    if args.weights:
        sd = torch.load(args.weights, map_location="cpu", weights_only=True)
        w = sd[args.layer + ".weight"].float()
    else:
        idx, spec = synthetic.find_layer(args.model_name, args.layer)
        w = torch.from_numpy(synthetic.layer_weight(spec, idx))
    if w.dim() == 4:   # intended reshape of scripts/factorize.py:140-147
        w = w.reshape(w.shape[0], w.shape[1]) if w.shape[2:] == (1, 1) else w.reshape(w.shape[0], w.shape[1], -1)
    if w.dim() not in (2, 3):
        raise ValueError('Incorrect number of dimentions in weight tensor')
    return w.to(device)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description="ADMM quantized CP factorization of one layer (MI355X)")
    ap.add_argument("--model-name", type=str, required=True, help="[resnet18, resnet50, llama7b]")
    ap.add_argument("--with-wandb", action="store_true",
                    help="log per-sweep metrics (JSONL at <outdir>/<prefix>_metrics.jsonl unless --metrics-jsonl)")
    ap.add_argument("--metrics-jsonl", type=str, default=None, help="per-sweep JSONL metrics file")
    ap.add_argument("--method", type=str, required=True, help="[admm, parafac, parafac-epc]")
    ap.add_argument("--init", type=str, default="random", help="[random, svd, parafac, parafac-epc]")
    ap.add_argument("--layer", type=str, required=True)
    ap.add_argument("--rank", type=int, required=False)
    ap.add_argument("--reduction-rate", type=float, required=False)
    ap.add_argument("--bits", type=int, required=True)
    ap.add_argument("--max_iter_als", type=int, default=5000)
    ap.add_argument("--max_iter_admm", type=int, default=1000)
    ap.add_argument("--max_iter_epc", type=int, default=5000)
    ap.add_argument("--seed", type=int, required=True)
    ap.add_argument("--qscheme", type=str, required=True)
    ap.add_argument("--weights", type=str, default=None, help="state_dict file (weights_only load); default synthetic")
    ap.add_argument("--outdir-root", type=str, default=".")
    args = ap.parse_args(argv)
    if args.rank is None and args.reduction_rate is None:
        raise ValueError('One of [--rank, --reduction-rate] arguments must be specified.')
    if args.method not in ['admm', 'parafac', 'parafac-epc']:
        raise ValueError('Method must be on of [admm, parafac, parafac-epc].')
    return args


def main(argv=None):
    if not torch.cuda.is_available():
        raise RuntimeError("admmq.factorize needs a ROCm GPU")
    device = torch.device("cuda:0")
    args = parse_args(argv)
    torch.manual_seed(args.seed)
    weight = _layer_weight(args, device)
    if args.rank is None:
        args.rank = int(weight.numel() / sum(list(weight.shape)) / args.reduction_rate)
    outdir = os.path.join(args.outdir_root, f'{args.bits}bit_{args.qscheme}/factors_{args.method}_seed{args.seed}')
    os.makedirs(outdir, exist_ok=True)
    fileprefix = f'{args.layer}_{args.method}_{args.init}_rank_{args.rank}'
    start = time.time()
    mpath = args.metrics_jsonl or (os.path.join(outdir, fileprefix + '_metrics.jsonl') if args.with_wandb else None)
    writer = JsonlWriter(mpath) if mpath else None
    if args.method == 'admm':
        try:
            run = factorize_layers([weight], [args.rank], args.max_iter_als, args.max_iter_admm, args.bits,
                                   args.qscheme, args.init, args.seed, names=[args.layer], metrics=writer)[0]
        finally:
            if writer is not None:
                writer.close()
        factors, factors_q = run.result()
        torch.save(run.loss, os.path.join(outdir, fileprefix + '_losshist.pt'))
        torch.save(run.lossq, os.path.join(outdir, fileprefix + '_lossquanthist.pt'))
    else:
        from .parafac_epc import parafac, parafac_epc
        if args.method == 'parafac':
            _, factors = parafac(weight, rank=args.rank, init=args.init, random_state=args.seed, tol=1e-8,
                                 n_iter_max=args.max_iter_als)
        else:
            _, factors = parafac_epc(weight, rank=args.rank, init=args.init, als_maxiter=args.max_iter_als,
                                     epc_maxiter=args.max_iter_epc)
        factors = [f.float().contiguous() for f in factors]
        factors_q = quantize_batched(factors, args.bits, args.qscheme)
    print('Factorization took {} minutes'.format((time.time() - start) / 60))
    for mode, factor in enumerate(factors):
        torch.save(factor.cpu(), os.path.join(outdir, fileprefix + f'_mode_{mode}.pt'))
    error, qerror = rel_error_batched([(weight, factors), (weight, factors_q)])
    print('Factorization error is {} for usual and {} for quantized'.format(error, qerror))
    return factors, factors_q


if __name__ == "__main__":
    main()

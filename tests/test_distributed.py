"""Multi-rank paths of bench.py on CPU with the gloo backend (world_size 2).

The GPU bench runs one process per GPU over RCCL; its data path has no collective
(every rank factorizes its own replica, or its LPT share of one model's layers) and
the only exchanges are the per-step factor gather and the max/sum timing reduction.
These run here on CPU tensors over gloo, with the same functions the bench calls.
"""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "admm-quantization_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, port, shard, q):
    try:
        import torch
        import torch.distributed as dist
        import bench
        from admmq import synthetic
        from admmq.factorize import LayerRun

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        dev = torch.device("cpu")
        work, numel, info = bench.build_workload("resnet18", rank, WORLD, shard, dev)
        names = [s.name for (s, _, _, _) in work]
        wsum = float(sum(W.double().sum() for (_, W, _, _) in work))
        runs = [LayerRun(s.name, W, R, [f.clone() for f in init]) for (s, W, R, init) in work]
        n_local = sum(f.numel() for r in runs for f in r.factors)
        assert numel[rank] == n_local   # the static shard plan knows every rank's size
        gathered = bench.gather_factors(runs, rank, WORLD, numel, dev)
        el, fi = bench.reduce_over_ranks(1.0 + rank, 100 * (rank + 1), WORLD, dev)
        specs = synthetic.MODELS["resnet18"]()
        dist.destroy_process_group()
        q.put((rank, names, wsum, n_local, gathered, el, fi, len(specs), info))
    except Exception as e:  # surfaced by the parent
        q.put((rank, "error", repr(e)))


def _run(shard):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, shard, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(WORLD):
        item = q.get(timeout=300)
        assert item[1] != "error", item
        out[item[0]] = item
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_replica_weak_scaling_gather():
    """Replica mode: every rank holds all 16 layers with its own weights (seeds
    1000 + l + 100 r); rank 0 gathers every rank's factors; the timing reduction is
    MAX over elapsed and SUM over factor-iterations."""
    out = _run("replica")
    r0, r1 = out[0], out[1]
    assert r0[1] == r1[1] and len(r0[1]) == r0[7] == 16
    assert r0[2] != r1[2]                      # different replica weights
    assert r0[4] == r1[4] == r0[3] + r1[3]     # gathered element count = all ranks' factors
    assert r0[5] == r1[5] == 2.0               # slowest rank's elapsed
    assert r0[6] == r1[6] == 300.0             # total factor-iterations


def test_layer_sharding_partitions_model():
    """--shard layers: the LPT split gives every layer to exactly one rank (same
    weights as the single-GPU run), and the gather still covers every factor."""
    out = _run("layers")
    r0, r1 = out[0], out[1]
    assert set(r0[1]).isdisjoint(r1[1])
    assert len(r0[1]) + len(r1[1]) == r0[7]
    assert r0[4] == r1[4] == r0[3] + r1[3]
    # the line's LPT cap: total cost over the busiest rank's, <= world and <= the whole-layer cap
    info = r0[8]
    assert info["layers_per_rank"] == [len(r0[1]), len(r1[1])]
    assert 1.0 < info["lpt_speedup_cap"] <= WORLD
    assert info["whole_layer_speedup_cap"] == pytest.approx(4.2, abs=0.1)   # resnet18


def test_lpt_balance():
    """LPT puts the heaviest layers first on the least-loaded rank: with 2 ranks the
    load gap is at most the largest single layer cost."""
    import bench
    from admmq import synthetic
    specs = synthetic.MODELS["resnet18"]()
    owner = bench.lpt(specs, 2)
    loads = [0.0, 0.0]
    for i, s in enumerate(specs):
        loads[owner[i]] += bench.layer_cost(s, s.rank())
    biggest = max(bench.layer_cost(s, s.rank()) for s in specs)
    assert abs(loads[0] - loads[1]) <= biggest
    with pytest.raises(KeyError):
        owner[len(specs)]


def _bench_cli(*args, env_extra=None, timeout=300):
    import json
    import subprocess
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


@pytest.mark.parametrize("model", ["resnet18", "resnet50"])
def test_bench_gpus_flag_launches_ranks(model):
    """`python bench.py --gpus 2` with no launcher starts 2 rank processes itself (torch.
    distributed.run as a child of a parent that never touches the GPU): the
    line reports the 2 ranks actually formed, and rank 0's single gather holds every
    rank's factors (checked element for element against each rank's own factors)."""
    rc, line, err = _bench_cli("--gpus", "2", "--cpu-dry-run", "--steps", "1", "--warmup", "1", "--model", model)
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2 and line["ranks_formed"] == 2
    assert line["gathered_elements"] == line["expected_elements"]
    assert line["rank_factors_match"] == [True, True]
    assert sum(line["layers_per_rank"]) == line["layers_total"] == (16 if model == "resnet18" else 48)


def test_bench_gpus_one_unchanged_and_mismatch_refused():
    """--gpus 1 runs in-process (no launcher); a --gpus that disagrees with the launcher's
    WORLD_SIZE exits non-zero instead of reporting the wrong rank count."""
    rc, line, err = _bench_cli("--gpus", "1", "--cpu-dry-run", "--steps", "1", "--warmup", "0")
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 1 and line["rank_factors_match"] == [True]
    rc, line, err = _bench_cli("--gpus", "4", "--cpu-dry-run", env_extra={"WORLD_SIZE": "2"})
    assert rc == 2 and line is None and "refusing" in err

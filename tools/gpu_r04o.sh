#!/bin/bash
# Round-4 session O: C4 rocprofv3 evidence, emulated 8-GPU shards on the final kernels, the
# RCCL path on hardware at N = 1, low-rank loop profile.
cd "$(dirname "$0")/.." || exit 1
bash tools/gpu_run.sh \
  "o_dist|300|python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 2 --warmup 1 --no-cpu-baseline --force-dist" \
  "o_emu18|400|python -u bench.py --emulate-world 8 --model resnet18 --steps 2 --warmup 1" \
  "o_emu50|500|python -u bench.py --emulate-world 8 --model resnet50 --steps 2 --warmup 1" \
  "o_lrprof|200|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/o_lr -o lr -- python3 tools/lowrank_bench.py --outer 6 --check -5 --svd-sample 0" \
  "o_clean|60|find gpurun_out/o_lr -name '*kernel_trace*' -delete; find gpurun_out/o_lr -name '*.db' -delete; du -sh gpurun_out" \
  "o_prof50|900|bash tools/profile.sh r04 resnet50"

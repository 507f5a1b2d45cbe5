cd /root/repo
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_reference.py -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/cfg_tests.log 2>&1; rc=$?; tail -3 gpurun_out/cfg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --model llama7b --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_llama_w.log 2>&1 || exit $?
python -c "
import json; d=json.loads([l for l in open('gpurun_out/bench_llama_w.log') if l.startswith('{')][-1]); print(round(d['value']), round(d['ms_per_step'],1), {k: round(v,1) for k,v in d['kernel_avg_us'].items()})"

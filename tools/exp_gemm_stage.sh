set -o pipefail
mkdir -p gpurun_out
for st in 3 1 2; do
  timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --gemm-stage $st > gpurun_out/r06w_bench_st$st.json 2> gpurun_out/r06w_bench_st$st.err || exit 1
done
export ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so
ADMMQ_GEMM_F32_STAGE=1 timeout -k 10 120 python -u tools/gemm_timeline.py --mode 0 --iters 6 > gpurun_out/r06w_gemm_c3m0_st1.txt 2>&1

#!/bin/bash
# Round-3 session M: phase breakdown of the persistent thin-factor loop (TRACE build).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ADMMQ_LIB=$PWD/tools/tracelib/libadmmq.so timeout -k 10 300 python -u tools/thin_loop_timeline.py \
  > gpurun_out/m_tl_r18.log 2>&1 || exit $?
cat gpurun_out/m_tl_r18.log
echo done

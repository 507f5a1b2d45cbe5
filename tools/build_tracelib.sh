#!/bin/bash
# Diagnostic build of libadmmq.so with the per-block timelines compiled in (TRACE=1),
# into tools/tracelib/ (ADMMQ_LIB=tools/tracelib/libadmmq.so selects it; never the product).
mkdir -p "$(dirname "$0")/tracelib"
cd "$(dirname "$0")/../admm-quantization_amd/csrc" || exit 1
make -j8 TRACE=1 OBJDIR=../../build/obj_trace ../../tools/tracelib/libadmmq.so OUT=../../tools/tracelib/libadmmq.so

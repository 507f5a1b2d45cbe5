#!/bin/bash
# Diagnostic A/B builds of libadmmq.so (never the product; ADMMQ_LIB=<dir>/libadmmq.so selects
# one, the ctypes route): tools/varlib_cur (this tree), tools/varlib_ns (fused finalize
# without per-group stores: ADMMQ_FIN_STREAM=0), tools/varlib_head (HEAD's sources from a
# worktree at /tmp/headwt, if present).
cd "$(dirname "$0")/../admm-quantization_amd/csrc" || exit 1
R=$(cd ../.. && pwd)
make -j8 OBJDIR=$R/build/obj_cur $R/tools/varlib_cur/libadmmq.so OUT=$R/tools/varlib_cur/libadmmq.so || exit 1
make -j8 EXTRA=-DADMMQ_FIN_STREAM=0 OBJDIR=$R/build/obj_ns $R/tools/varlib_ns/libadmmq.so OUT=$R/tools/varlib_ns/libadmmq.so || exit 1
if [ -d /tmp/headwt/admm-quantization_amd/csrc ]; then
  make -C /tmp/headwt/admm-quantization_amd/csrc -j8 OBJDIR=/tmp/headwt/build/obj OUT=$R/tools/varlib_head/libadmmq.so \
    $R/tools/varlib_head/libadmmq.so || exit 1
fi

#!/bin/bash
# Builds the product library (gfx950) and the oracle checker library.
# The HIP translation units compile in parallel (one hipcc per unit), then link.
set -e
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
CSRC=dyros_robot_controller_amd/csrc
OBJ=build/obj${DRC_VARIANT:+_$DRC_VARIANT}
OUT=${DRC_OUT:-dyros_robot_controller_amd/libdrc_amd.so}
mkdir -p "$OBJ"
# -disable-machine-licm: the persistent instance loops would otherwise get the
# FP64 constants of the math library and the stages hoisted into registers at
# kernel entry, spilled to scratch and reloaded (from beyond L2) per instance
# -ffp-contract=on: a*b+c is fused only within one source expression, decided
# before inlining, so a device function rounds the same in every kernel it is
# inlined into -- the fused kernel and the two-kernel pipeline (and hence any
# batch size and sub-batch split) return bit-identical results
# (tests/test_gpu_fused.py, tests/test_gpu_dist.py).  Measured equal speed
# to the default (fast) contraction (profiles/r04c_ab_fpon.jsonl).
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -ffp-contract=on -mllvm -disable-machine-licm $DRC_EXTRA_FLAGS"
# build id (drc_build_id()): hash of the library's sources and flags, so a
# profiles/ counter summary can be matched to the build it was measured on
# (bench.py ignores summaries of another build)
# (and of the toolchain: the same sources built by another hipcc / ROCm are another build)
BUILD_ID=$(cat $CSRC/*.hip $CSRC/*.hpp $CSRC/*.cpp include/drc_amd.h include/drc_amd_debug.h build.sh | { cat; echo "$FLAGS"; $HIPCC --version 2>&1; } | sha256sum | cut -c1-16)
pids=()
for src in task_kernel.hip qp_kernel.hip fused_kernel.hip qpid_kernel.hip dynamics.hip order_kernel.hip api.cpp model.cpp; do
  XF=""
  [ "$src" = api.cpp ] && XF="-DDRC_BUILD_ID=\"$BUILD_ID\""
  $HIPCC $FLAGS $XF -c $CSRC/$src -o "$OBJ/${src%.*}.o" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
[ $rc -eq 0 ] || { echo "build.sh: a HIP translation unit failed to compile" >&2; exit 1; }
$HIPCC --offload-arch=gfx950 -shared -fPIC "$OBJ"/task_kernel.o "$OBJ"/qp_kernel.o "$OBJ"/fused_kernel.o "$OBJ"/qpid_kernel.o \
  "$OBJ"/dynamics.o "$OBJ"/order_kernel.o "$OBJ"/api.o "$OBJ"/model.o -o "$OUT" -Wl,-rpath,/opt/rocm/lib
[ -n "$DRC_VARIANT" ] && exit 0
# test-only: the narrow-phase device code on one wave per pair (tests/test_gpu_narrow.py)
$HIPCC $FLAGS -shared tests/gpu_narrow.hip -o tests/_narrow_gpu.so
make -s -C oracle all count
mkdir -p dyros_robot_controller_amd/python
# C++ facade + pybind11 module with the reference's module/class names (host code only)
PYEXT=$(python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYINC=$(python3 -c "import pybind11, sysconfig; print('-I' + pybind11.get_include() + ' -I' + sysconfig.get_paths()['include'])")
g++ -O2 -std=c++17 -shared -fPIC -Wall $PYINC -Iinclude \
  dyros_robot_controller_amd/cpp/bindings.cpp -o dyros_robot_controller_amd/python/dyros_robot_controller_cpp_wrapper$PYEXT \
  -Ldyros_robot_controller_amd -ldrc_amd -Wl,-rpath,'$ORIGIN/..'

#!/bin/bash
# Diagnostic builds: task-kernel occupancy variants and the phase-timing build.
set -e
cd "$(dirname "$0")/.."
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SRC="dyros_robot_controller_amd/csrc/qpik_kernel.hip dyros_robot_controller_amd/csrc/dynamics.hip dyros_robot_controller_amd/csrc/model.cpp"
for w in ${WAVES:-1 2 3 4}; do
  $HIPCC --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -DDRC_TASK_WAVES=$w $SRC \
    -o dyros_robot_controller_amd/libdrc_amd_w$w.so -Wl,-rpath,/opt/rocm/lib &
done
$HIPCC --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -DDRC_PHASE_TIMING $SRC \
  -o dyros_robot_controller_amd/libdrc_amd_timing.so -Wl,-rpath,/opt/rocm/lib &
wait

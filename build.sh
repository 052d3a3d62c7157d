#!/bin/bash
# Builds the product library (gfx950) and the oracle checker library.
set -e
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
$HIPCC --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -Wall -Wno-unused-function \
  dyros_robot_controller_amd/csrc/qpik_kernel.hip dyros_robot_controller_amd/csrc/model.cpp \
  -o dyros_robot_controller_amd/libdrc_amd.so -Wl,-rpath,/opt/rocm/lib
make -s -C oracle

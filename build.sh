#!/bin/bash
# Builds the product library (gfx950) and the oracle checker library.
set -e
cd "$(dirname "$0")"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
$HIPCC --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -Wall -Wno-unused-function \
  dyros_robot_controller_amd/csrc/qpik_kernel.hip dyros_robot_controller_amd/csrc/dynamics.hip dyros_robot_controller_amd/csrc/model.cpp \
  -o dyros_robot_controller_amd/libdrc_amd.so -Wl,-rpath,/opt/rocm/lib
make -s -C oracle
mkdir -p dyros_robot_controller_amd/python
# C++ facade + pybind11 module with the reference's module/class names (host code only)
PYEXT=$(python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYINC=$(python3 -c "import pybind11, sysconfig; print('-I' + pybind11.get_include() + ' -I' + sysconfig.get_paths()['include'])")
g++ -O2 -std=c++17 -shared -fPIC -Wall $PYINC -Iinclude \
  dyros_robot_controller_amd/cpp/bindings.cpp -o dyros_robot_controller_amd/python/dyros_robot_controller_cpp_wrapper$PYEXT \
  -Ldyros_robot_controller_amd -ldrc_amd -Wl,-rpath,'$ORIGIN/..'

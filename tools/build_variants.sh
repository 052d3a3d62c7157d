#!/bin/bash
# Diagnostic builds through build.sh: task-kernel occupancy variants
# (WAVES="1 2 3 4") and the phase-timing build (libdrc_amd_timing.so).
set -e
cd "$(dirname "$0")/.."
for w in ${WAVES:-}; do
  DRC_VARIANT=w$w DRC_EXTRA_FLAGS="-DDRC_TASK_WAVES=$w" DRC_OUT=dyros_robot_controller_amd/libdrc_amd_w$w.so bash build.sh
done
DRC_VARIANT=timing DRC_EXTRA_FLAGS="-DDRC_PHASE_TIMING" DRC_OUT=dyros_robot_controller_amd/libdrc_amd_timing.so bash build.sh

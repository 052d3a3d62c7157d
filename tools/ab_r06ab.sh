# r06ab: phase timing of UR5e / XLS-FR3 on the current kernels; FETCH_SIZE calibration at 4 / 8 / 16 B per lane
set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/phase_timing.py ur5e > gpurun_out/r06ab_phase_ur5e.txt 2>&1
timeout -k 10 200 python3 tools/phase_timing.py xls_fr3 > gpurun_out/r06ab_phase_xls_fr3.txt 2>&1
OUT=$GRAFT_REPO_ROOT/gpurun_out/fetch_calib_r06ab
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o fetch -- $GRAFT_REPO_ROOT/tools/fetch_calib > $OUT/fetch.log 2>&1
echo "calibration pass done"
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06ab_smoke.log 2>&1

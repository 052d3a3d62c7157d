cd /tmp; export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/occ
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/a -o a -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/a.log 2>&1
echo rc $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU -f csv -d $O/b -o b -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/b.log 2>&1
echo rc $?

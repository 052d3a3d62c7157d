# r06z: fusion up to 16 384 for every compiled shape (manipulators ordered): GPU suite + bench lines
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu_suite.sh r06z
for b in 4096 12288 16384; do for r in fr3 ur5e xls_fr3; do echo "$r $b: $(timeout -k 10 300 python3 bench.py --robot $r --batch $b --no-cpu-baseline --no-extras --steps 20 --warmup 5 | cut -c90-130)"; done; done
echo "husky_fr3 16384: $(timeout -k 10 300 python3 bench.py --robot husky_fr3 --no-cpu-baseline --no-extras --steps 20 --warmup 5 | cut -c90-130)"

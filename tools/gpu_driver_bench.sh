# The driver's exact bench command on the current tree, with its wall time.
# usage: bash tools/gpu_driver_bench.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; T=$1
cd $R && mkdir -p gpurun_out
s=$(date +%s.%N)
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_driver_bench.log 2>&1 || { tail -n 30 gpurun_out/${T}_driver_bench.log; exit 1; }
e=$(date +%s.%N)
echo "wall_s $(python3 -c "print(round($e-$s,1))")" | tee -a gpurun_out/${T}_driver_bench.log
tail -n 2 gpurun_out/${T}_driver_bench.log

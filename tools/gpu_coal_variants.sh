# Per coalesce variant (tools/build_coal_variants.sh): parity tests, phase clocks, TB bench line.
# usage: bash tools/gpu_coal_variants.sh <tag> "t1024p6 t512p8 ..."
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R && mkdir -p gpurun_out
TAG=$1
for v in $2; do
  export DQRM_LIB_PATH=$R/tools/diag_build/libdqrm_$v.so
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "criteo_form_coalesce or dp_ or pool1 or kaggle or terabyte or tb_" > gpurun_out/${TAG}_${v}_tests.log 2>&1 || { echo "$v TESTS FAIL"; tail -n 30 gpurun_out/${TAG}_${v}_tests.log; exit 1; }
  echo "$v $(tail -n 1 gpurun_out/${TAG}_${v}_tests.log)"
  DQRM_LIB_PATH=$R/tools/diag_build/libdqrm_${v}_clock.so timeout -k 10 120 python tools/diag_coalesce.py terabyte > gpurun_out/${TAG}_${v}_diag.log 2>&1 || { tail gpurun_out/${TAG}_${v}_diag.log; exit 1; }
  head -n 8 gpurun_out/${TAG}_${v}_diag.log | tail -n 7; tail -n 2 gpurun_out/${TAG}_${v}_diag.log
  timeout -k 10 300 python bench.py --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 > gpurun_out/${TAG}_${v}_bench.log 2>&1 || { tail -n 20 gpurun_out/${TAG}_${v}_bench.log; exit 1; }
  tail -n 1 gpurun_out/${TAG}_${v}_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('BENCH', d['value'], d['us_per_step'], d['kernels_ms'], d['roofline']['avg_launch_ms'])"
done

# Round-5: k_sgd_small narrow-table W staging (config 3) A/B, the DLRM config-3 line with the
# presummed vs per-lookup sparse grad, and TCC request counters of the Kaggle one-launch kernel
# + known-byte calibration (verdict item 6).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r5i}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread \
    > gpurun_out/${T}_tests.log 2>&1 || { tail -n 40 gpurun_out/${T}_tests.log; exit 1; }
tail -n 2 gpurun_out/${T}_tests.log
C3="--config kaggle --batch-per-gpu 128 --mode sgd --steps 400 --warmup 40 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0"
for round in 1 2; do
for v in "wl||$C3" "nowl|DQRM_SG_WLDS=0|$C3" "wlg||$C3 --graph --graph-steps 32" "nowlg|DQRM_SG_WLDS=0|$C3 --graph --graph-steps 32"; do
  lab=${v%%|*}; rest=${v#*|}; envs=${rest%%|*}; args=${rest#*|}
  env $envs timeout -k 10 300 python -u bench.py $args > gpurun_out/${T}_${lab}_$round.log 2>&1 || { tail -n 20 gpurun_out/${T}_${lab}_$round.log; exit 1; }
  tail -n 1 gpurun_out/${T}_${lab}_$round.log >> gpurun_out/${T}_lines.jsonl
  tail -n 1 gpurun_out/${T}_${lab}_$round.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('$lab', d['us_per_step'], d.get('kernels_ms'))"
done
done
# rocprof kernel trace of both c3 forms
for v in "wl|" "nowl|DQRM_SG_WLDS=0"; do
  lab=${v%%|*}; envs=${v#*|}
  (cd /tmp && env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_c3$lab -o tb --output-format csv -- python3 $R/bench.py $C3 > $R/gpurun_out/prof_${T}_c3$lab.log 2>&1) || { tail -n 20 gpurun_out/prof_${T}_c3$lab.log; exit 1; }
  python3 tools/kmedian.py gpurun_out/prof_${T}_c3$lab sgd_small
done
timeout -k 10 300 python -u tools/diag_sgd.py 128 > gpurun_out/${T}_phase_sgd.txt 2>&1 || { tail -n 20 gpurun_out/${T}_phase_sgd.txt; exit 1; }
head -n 8 gpurun_out/${T}_phase_sgd.txt
# DLRM config 3: unchanged list + torch SGD, presummed (default) vs per-lookup COO
DL="--mode dlrm --config kaggle --batch-per-gpu 128 --dropin-form list --grad-mode sparse --steps 100 --warmup 10 --cpu-baseline 0"
for v in "presum|DQRM_SPARSE_GRAD=presummed" "perlookup|DQRM_SPARSE_GRAD=per_lookup"; do
  lab=${v%%|*}; envs=${v#*|}
  env $envs timeout -k 10 400 python -u bench.py $DL > gpurun_out/${T}_dlrm_$lab.log 2>&1 || { tail -n 20 gpurun_out/${T}_dlrm_$lab.log; exit 1; }
  tail -n 1 gpurun_out/${T}_dlrm_$lab.log >> gpurun_out/${T}_dlrm_lines.jsonl
  tail -n 1 gpurun_out/${T}_dlrm_$lab.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('dlrm $lab', d['us_per_step'], d['torch_gpu_reference']['us_per_step'])"
done
# TCC request counters: list, Kaggle one-launch step, calibration on known bytes
(cd /tmp && timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/${T}_counters.txt 2>&1) || { tail -n 5 gpurun_out/${T}_counters.txt; exit 1; }
grep -o "TCC_EA0_[A-Z0-9_]*" gpurun_out/${T}_counters.txt | sort -u | tr '\n' ' '; echo
python3 tools/pmc_tcc.py ${T}_kaggle gpurun_out/${T}_counters.txt -- python3 $R/bench.py --config kaggle --steps 20 --warmup 5 --cpu-baseline 0 --gather-batch 0 --mlp-iters 0 > gpurun_out/${T}_tcc_kaggle.txt 2>&1 || { tail -n 5 gpurun_out/${T}_tcc_kaggle.txt; exit 1; }
grep -i "coalesce\|index\|pass" gpurun_out/${T}_tcc_kaggle.txt | head -n 30
python3 tools/pmc_tcc.py ${T}_calib gpurun_out/${T}_counters.txt -- python3 $R/tools/pmc_calib.py > gpurun_out/${T}_tcc_calib.txt 2>&1 || { tail -n 5 gpurun_out/${T}_tcc_calib.txt; exit 1; }
head -n 40 gpurun_out/${T}_tcc_calib.txt

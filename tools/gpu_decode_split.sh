# rocprofv3 kernel trace of one decode_suite case, split per step (tools/rocpd_split.py):
#   M=gptj|neox|bloom8 B=<batch> DT=bf16|fp16 bash tools/gpu_decode_split.sh
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
T=${M:-gptj}_b${B:-1}_${DT:-bf16}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/split_$T -o tr -- python3 $R/bench/decode_suite.py --models ${M:-gptj} --batches ${B:-1} --dtypes ${DT:-bf16} > $R/gpurun_out/split_$T.log 2>&1 || exit 1
db=$(find $R/gpurun_out/split_$T -name "*.db" | head -1)
python3 $R/tools/rocpd_split.py "$db" --last-steps 10 --step-kernel sample_ > $R/gpurun_out/split_$T.txt
rm -rf $R/gpurun_out/split_$T

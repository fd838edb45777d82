# GPU job: kernel-level profile of the PTQ runs (where does the non-GEMM time go?).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ptq_fp8 -o run -- python scripts/ptq_llama.py --no-baseline > gpurun_out/prof_ptq_fp8.json 2> gpurun_out/prof_ptq_fp8.err || exit 21
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ptq_awq -o run -- python scripts/ptq_llama.py --config INT4_AWQ_CFG --samples 64 --no-baseline > gpurun_out/prof_ptq_awq.json 2> gpurun_out/prof_ptq_awq.err || exit 22
find gpurun_out/prof_ptq_fp8 gpurun_out/prof_ptq_awq -name "*kernel_stats.csv" > gpurun_out/prof_files.txt

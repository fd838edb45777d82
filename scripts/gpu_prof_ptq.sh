# GPU job: kernel-level profile of the PTQ runs (where does the non-GEMM time go?).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ptq_fp8" -o run --output-format csv -- python3 "$R/benchmarks/ptq_llama.py" --no-baseline > "$R/gpurun_out/prof_ptq_fp8.json" 2> "$R/gpurun_out/prof_ptq_fp8.err" || exit 21
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ptq_awq" -o run --output-format csv -- python3 "$R/benchmarks/ptq_llama.py" --config INT4_AWQ_CFG --samples 64 --no-baseline > "$R/gpurun_out/prof_ptq_awq.json" 2> "$R/gpurun_out/prof_ptq_awq.err" || exit 22
find "$R/gpurun_out/prof_ptq_fp8" "$R/gpurun_out/prof_ptq_awq" -type f ! -name "*stats.csv" -delete
find "$R/gpurun_out/prof_ptq_fp8" "$R/gpurun_out/prof_ptq_awq" -name "*stats.csv" > "$R/gpurun_out/prof_files.txt"

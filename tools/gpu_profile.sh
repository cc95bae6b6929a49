set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
cd $R
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_r1_bench.json 2> $R/gpurun_out/prof_r1.err
echo PROF_EXIT $?
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pmc_fetch_r1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile > $R/gpurun_out/pmc_fetch.json 2> $R/gpurun_out/pmc_fetch.err
echo PMC1_EXIT $?
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pmc_write_r1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile > $R/gpurun_out/pmc_write.json 2> $R/gpurun_out/pmc_write.err
echo PMC2_EXIT $?
find $R/gpurun_out -name "*.csv" | head -20

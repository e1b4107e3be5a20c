set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 50 --warmup 5 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
echo "bench rc=$?"
cat gpurun_out/bench1.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/prof1.log 2>&1
echo "prof rc=$?"
find gpurun_out/prof1 -name "*stats*"

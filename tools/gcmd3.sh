# full GPU suite, smoke, N=1 bench, rocprof passes of the N=1 bench (round 5 final-code check)
rm -f gpurun_out/steps.log
S=tools/gpu_step.sh
$S tests 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread || exit 1
$S smoke 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S n1 200 python bench.py || exit 1
PROF_TAG=r05 $S prof 900 bash tools/profile_reduce.sh || exit 1
cat gpurun_out/steps.log

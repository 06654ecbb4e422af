# Eager vs graph replay (bench.py --launch) at 20 and 200 timed steps, two rounds, after the graph/prefetch tests.
set -e
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_prefetch.py > gpurun_out/graph_tests.log 2>&1
for r in 1 2; do
for L in eager graph; do
for K in 20 200; do
timeout -k 10 200 python bench.py --steps $K --warmup 5 --launch $L --no-cpu-baseline --fp32-steps 0 --bf16-steps 0 --no-data-path --no-parity > gpurun_out/lg_${L}_${K}_$r.log 2>&1
python -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/lg_${L}_${K}_$r.log') if l.startswith('{')][0]; print('$L K=$K r$r', round(d['ms_per_step']*1e3,1), 'us', d['launch'])"
done; done; done

#!/bin/bash
# Round-6 check call: the 2-rank bench rehearsal test (node pass), the b76 stress against the Montgomery form, and
# the driver's bench command once more (another box).
T=${1:-r06r}
mkdir -p gpurun_out
bash tools/gpu.sh $T test:tests/test_gpu_bench_rehearse.py test:tests/test_integration_shim.py test:tests/test_gpu_parity.py || exit 1
timeout -k 10 300 python tools/b76_stress.py 2097152 2 > gpurun_out/${T}_b76_stress.json 2> gpurun_out/${T}_b76_stress.err \
  || { echo "b76 stress failed"; cat gpurun_out/${T}_b76_stress.json; tail -5 gpurun_out/${T}_b76_stress.err; exit 1; }
cat gpurun_out/${T}_b76_stress.json
bash tools/gpu.sh $T bench:--steps,20,--warmup,5

#!/bin/bash
# Round-6 measurement call: fresh PMC of the exponentiation (enc) and merge (kway) workloads, the whole GPU suite,
# smoke, the driver's bench command and its rocprof kernel trace (tools/gpu.sh steps).
T=${1:-r06q}
bash tools/gpu.sh $T pmc:enc pmc:kway suite smoke bench:--steps,20,--warmup,5 trace

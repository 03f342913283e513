#!/bin/bash
# Round-6 add-kernel check: its GPU tests and configs[3], the A/B against the round-5 library, fresh add / merge PMC.
T=${1:-r06t}
bash tools/gpu.sh $T test:tests/test_gpu_addb.py test:tests/test_gpu_configs.py test:tests/test_integration_shim.py || exit 1
bash tools/addb_lib_ab.sh $T tools/bin/libfthe_r05.so || exit 1
bash tools/gpu.sh $T pmc:add pmc:addsame pmc:kway opstrace

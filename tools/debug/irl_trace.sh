#!/bin/bash
# Build the irl step trace library (kernels/irl.hip with -DZR_IRL_TRACE, linked with the product's
# other objects from build/obj) into tools/debug/trace_lib/ -- a debug build, never loaded by the
# product, the tests or bench.py.  Run the trace with tools/debug/irl_trace.py on the GPU box.
set -e
cd "$(dirname "$0")/../.."
OBJ=build/obj
mkdir -p build/trace tools/debug/trace_lib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fhip-fp32-correctly-rounded-divide-sqrt -DZR_IRL_TRACE -c zaru_amd/csrc/kernels/irl.hip -o build/trace/k_irl.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o tools/debug/trace_lib/libzaru_hip.so \
  $(ls $OBJ/k_*.o $OBJ/r_*.o | grep -v '/k_irl.o$') build/trace/k_irl.o -Wl,-soname,libzaru_hip.so -L/opt/rocm/lib -lrccl
echo "built tools/debug/trace_lib/libzaru_hip.so"

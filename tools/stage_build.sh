#!/bin/bash
# Build the libraries into build/stage (not shipped to the GPU box) and, with "install", move them
# into zaru_amd/lib by rename -- so a gpurun snapshot taken meanwhile never sees a half-written .so.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/stage
make -s -j8 -C zaru_amd/csrc LIBDIR=../../build/stage
if [ "$1" = "install" ]; then
  for f in build/stage/libzaru_hip.so build/stage/_zaru_host*.so; do mv -f "$f" zaru_amd/lib/; done
  echo "installed"
fi

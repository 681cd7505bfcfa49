#!/bin/bash
# Build tools/batch_bench against the in-tree lib0xfec_hip.so (hipcc, gfx950 host code only).
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
ROOT="$(dirname "$HERE")"
/opt/rocm/bin/hipcc -O2 -std=c++17 -o "$HERE/batch_bench" "$HERE/batch_bench.cpp" \
  -L"$ROOT/0xfec_amd" -l0xfec_hip -Wl,-rpath,"\$ORIGIN/../0xfec_amd"

#!/bin/bash
# Builds variants of the library with other large-universe kernel shapes (COOC_SP_THREADS,
# COOC_SP_TSHIFT) as csrc/libcooc_hip_<name>.so for A/B runs (scripts/bench_c3.py --lib).
set -e
cd "$(dirname "$0")/.."
build() {  # name threads tshift
  B=/tmp/cooc_var_$1
  rm -rf $B && mkdir -p $B/flink-cooccurrence_amd && cp -r flink-cooccurrence_amd/csrc $B/flink-cooccurrence_amd/ && cp -r include $B/
  rm -f $B/flink-cooccurrence_amd/csrc/*.o $B/flink-cooccurrence_amd/csrc/*.so
  make -s -j8 -C $B/flink-cooccurrence_amd/csrc CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fvisibility=hidden -fvisibility-inlines-hidden -DCOOC_SP_THREADS=$2 -DCOOC_SP_TSHIFT=$3 $4" >/dev/null
  cp $B/flink-cooccurrence_amd/csrc/libcooc_hip.so flink-cooccurrence_amd/csrc/libcooc_hip_$1.so
}
for v in "$@"; do build $v; done

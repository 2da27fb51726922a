#!/bin/bash
# Builds the per-workgroup phase-statistics variant of the library (COOC_SP_STATS) next to the
# release one, as csrc/libcooc_hip_stats.so (the release .so is untouched).
set -e
cd "$(dirname "$0")/.."
B=/tmp/cooc_stats_build
rm -rf $B && mkdir -p $B/flink-cooccurrence_amd && cp -r flink-cooccurrence_amd/csrc $B/flink-cooccurrence_amd/ && cp -r include $B/ && rm -f $B/flink-cooccurrence_amd/csrc/*.o $B/flink-cooccurrence_amd/csrc/*.so
make -s -j8 -C $B/flink-cooccurrence_amd/csrc CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fvisibility=hidden -fvisibility-inlines-hidden -DCOOC_SP_STATS" >/dev/null
cp $B/flink-cooccurrence_amd/csrc/libcooc_hip.so flink-cooccurrence_amd/csrc/libcooc_hip_stats.so

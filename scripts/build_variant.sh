#!/bin/bash
# Builds a variant of the library from the working tree (extra compile flags in $2) as
# flink-cooccurrence_amd/csrc/libcooc_hip_$1.so, leaving the release build untouched.  Use with COOC_LIB=.
set -e
cd "$(dirname "$0")/.."
B=/tmp/cooc_variant_$1
rm -rf $B && mkdir -p $B/flink-cooccurrence_amd && cp -r flink-cooccurrence_amd/csrc $B/flink-cooccurrence_amd/ && cp -r include $B/
rm -f $B/flink-cooccurrence_amd/csrc/*.o $B/flink-cooccurrence_amd/csrc/*.so
make -s -j8 -C $B/flink-cooccurrence_amd/csrc CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -fvisibility=hidden -fvisibility-inlines-hidden ${2:-}" >/dev/null 2>&1
cp $B/flink-cooccurrence_amd/csrc/libcooc_hip.so flink-cooccurrence_amd/csrc/libcooc_hip_$1.so
echo built flink-cooccurrence_amd/csrc/libcooc_hip_$1.so

#!/bin/bash
# Builds tests/sanitize/stream_asan: the library with AddressSanitizer + UndefinedBehaviorSanitizer on its HOST
# code (each -fsanitize behind -Xarch_host; the kernels are built as in the release library, GPU sanitizers
# being unavailable) linked with tests/sanitize/stream_driver.cpp.  Runs on a GPU box
# (tests/test_stream_asan_gpu.py).  The release library is untouched.
set -e
cd "$(dirname "$0")/.."
B=$(mktemp -d "${TMPDIR:-/tmp}/cooc_asan_build.XXXXXX")  # per invocation: concurrent builds do not collide
trap 'rm -rf "$B"' EXIT
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all -Xarch_host -fno-omit-frame-pointer -Xarch_host -g"
mkdir -p $B/flink-cooccurrence_amd && cp -r flink-cooccurrence_amd/csrc $B/flink-cooccurrence_amd/ && cp -r include $B/ \
  && rm -f $B/flink-cooccurrence_amd/csrc/*.o $B/flink-cooccurrence_amd/csrc/*.so
make -s -j${MAKE_JOBS:-8} -C $B/flink-cooccurrence_amd/csrc CXXFLAGS="-O2 -std=c++17 -fPIC -Wall -Wno-unused-result $SAN" \
  cooc_count.o cooc_sparse.o cooc_verify.o cooc_stream_k.o cooc_shard.o cooc_owned.o cooc_stream.o cooc_ctx.o \
  cooc_capi.o cooc_comm.o cooc_codec.o cooc_ingest.o >/dev/null
/opt/rocm/bin/hipcc -O1 -std=c++17 $SAN -Iinclude -c -o $B/stream_driver.o tests/sanitize/stream_driver.cpp
/opt/rocm/bin/hipcc --offload-arch=gfx950 $SAN -o tests/sanitize/stream_asan $B/stream_driver.o \
  $B/flink-cooccurrence_amd/csrc/*.o -ldl
echo "built tests/sanitize/stream_asan"

#!/bin/sh
# Builds tools/latency (single-record GPU CipherState latency, tools/latency.c)
# tools/mt_calls (single-call throughput over threads, tools/mt_calls.c) and
# tools/queue_probe (other streams beside resident workers, tools/queue_probe.cpp)
# and tools/wire_bench (the end-to-end wire path timed from C, tools/wire_bench.c).
set -e
cd "$(dirname "$0")/.."
gcc -O2 -Iinclude tools/latency.c -Lnoise-c_amd/lib -lnoise_aead_hip \
    -Wl,-rpath,'$ORIGIN/../noise-c_amd/lib' -o tools/latency
gcc -O2 -pthread -Iinclude tools/mt_calls.c -Lnoise-c_amd/lib -lnoise_aead_hip \
    -Wl,-rpath,'$ORIGIN/../noise-c_amd/lib' -o tools/mt_calls
/opt/rocm/bin/hipcc -O2 -std=c++17 -Iinclude tools/queue_probe.cpp -Lnoise-c_amd/lib -lnoise_aead_hip \
    -Wl,-rpath,'$ORIGIN/../noise-c_amd/lib' -lpthread -o tools/queue_probe
gcc -O2 -std=c11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tools/wire_bench.c -Lnoise-c_amd/lib \
    -lnoise_aead_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$ORIGIN/../noise-c_amd/lib' -Wl,-rpath,/opt/rocm/lib \
    -o tools/wire_bench

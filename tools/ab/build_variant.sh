#!/bin/sh
# Rebuild an A/B variant of the library from the sources of a git revision
# (round 6, VERDICT r5 item 8: the shipped kernels keep one body each; the
# A/B arms of rounds 1-5 live in the history — tools/ab/README.md lists each
# DESIGN.md record with its revision and defines).
#
#   sh tools/ab/build_variant.sh NAME REV "DEFS"
#     -> noise-c_amd/ab/libnoise_aead_hip_NAME.so (NOISE_AEAD_LIB=... selects it;
#        tools/gpu/run.sh's `ab` step takes NAME)
#
# e.g. sh tools/ab/build_variant.sh authreg4 ab-arms-r5 "-DNA_AUTH_REG=4"
set -eu
NAME=$1 REV=$2 DEFS=${3:-}
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
TMP=$(mktemp -d /tmp/nab.XXXXXX)
trap 'rm -rf "$TMP"' EXIT
git -C "$ROOT" archive "$REV" include noise-c_amd | tar -x -C "$TMP"
make -s -C "$TMP/noise-c_amd" variant NAME="$NAME" DEFS="$DEFS"
mkdir -p "$ROOT/noise-c_amd/ab"
cp "$TMP/noise-c_amd/ab/libnoise_aead_hip_$NAME.so" "$ROOT/noise-c_amd/ab/"
echo "built noise-c_amd/ab/libnoise_aead_hip_$NAME.so from $REV ($DEFS)"

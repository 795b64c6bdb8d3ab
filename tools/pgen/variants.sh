#!/bin/bash
# Build alternative generated code objects for A/B timing (PA_GEN_DIR=...):
#   tools/pgen/variants.sh NAME [ENV=VAL ...]  -> gpuvar/NAME/*.hsaco
# The non-default kernels are copied from pairing_amd/lib.
set -e
cd "$(dirname "$0")/../.."
name=$1; shift
out=gpuvar/$name
mkdir -p $out
cp pairing_amd/lib/pa_gen_*.hsaco $out/
env "$@" python3 tools/pgen/build_gen.py ml fe --outdir $out

#!/bin/bash
# The library's build id: the first 16 hex digits of the SHA-256 of every
# source liblcfir.so is built from (csrc/*.hpp, csrc/*.hip in byte order, then
# include/lcfir.h).  The Makefile compiles it into the library
# (lcfir_build_id()); bench.py attaches a PMC sidecar only when the sidecar
# carries the loaded library's id; scripts/build_variant.sh stamps a variant
# with its base tree's id and scripts/gpu_run.sh refuses a variant whose base
# is not the tree it runs in.
# usage: src_hash.sh [PKG_DIR]   (default: this script's directory)
set -euo pipefail
D="${1:-$(cd "$(dirname "$0")" && pwd)}"
cd "$D"
cat $(ls csrc/*.hpp csrc/*.hip | LC_ALL=C sort) ../include/lcfir.h | sha256sum | cut -c1-16

#!/bin/bash
# Build a k_vsd compile-time variant for A/B runs (tools/variants.sh):
#   bash tools/mkvar.sh NAME "-DFLAG=VALUE ..."  ->  bop_toolkit_amd/lib/variants/NAME.so
set -e
cd "$(dirname "$0")/../bop_toolkit_amd/csrc"
make -s -j8 BUILD=build_var_$1 OUT=../lib/variants/$1.so EXTRA="$2"

#!/bin/bash
# Build libbopx.so of a git revision as an A/B variant:
#   bash tools/mkvar_rev.sh REV NAME ["-DFLAG=..."]  ->  bop_toolkit_amd/lib/variants/NAME.so
set -e
cd "$(dirname "$0")/.."
src=bop_toolkit_amd/csrc_rev_$2
rm -rf "$src"; mkdir -p "$src"
git archive "$1" bop_toolkit_amd/csrc | tar -x -C "$src" --strip-components=2
make -s -j8 -C "$src" BUILD=build OUT=../lib/variants/$2.so IO_OUT=../lib/variants/io_unused.so EXTRA="$3" ../lib/variants/$2.so
rm -rf "$src"

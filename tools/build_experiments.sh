#!/bin/bash
# The experiment build of libngz: the same sources with -DNGZ_EXPERIMENTS, so the knobs of
# ngz_knobs.cpp (NGZ_LDS, NGZ_LD_AUX, NGZ_AGG_GRID, ...) are read from the environment for A/B
# measurements.  Output: tools/exp/libngz_exp.so (outside the package, and listed in .gpurunignore:
# remove that line for a GPU run that needs it), loaded by the Python binding only when
# NGZ_EXPERIMENTS=1, with a warning on stderr.  The product library (libngz.so, __graft_entry__.build) reads no knobs.
# A compile-time variant: VARIANT=name DEFS="-DX=1 ..." -> libngz_exp_name.so (NGZ_EXPERIMENTS=name).
set -e
cd "$(dirname "$0")/.."
python3 -c "import sys; sys.path.insert(0, 'tools'); import embed_sources; embed_sources.main()"
mkdir -p tools/exp
OUT=tools/exp/libngz_exp${VARIANT:+_$VARIANT}.so
python3 -c "import __graft_entry__ as g, sys; g._build_lib('$OUT', ['-DNGZ_EXPERIMENTS'] + sys.argv[1:])" $DEFS

#!/bin/bash
# The experiment build of libngz: the same sources with -DNGZ_EXPERIMENTS, so the knobs of
# ngz_knobs.cpp (NGZ_LDS, NGZ_LD_AUX, NGZ_AGG_GRID, ...) are read from the environment for A/B
# measurements.  Output: netgauze_amd/libngz_exp.so, loaded by the Python binding only when
# NGZ_EXPERIMENTS=1.  The product library (libngz.so, __graft_entry__.build) reads no knobs.
set -e
cd "$(dirname "$0")/.."
python3 -c "import sys; sys.path.insert(0, 'tools'); import embed_sources; embed_sources.main()"
python3 -c "import __graft_entry__ as g; g._build_lib('netgauze_amd/libngz_exp.so', ['-DNGZ_EXPERIMENTS'])"

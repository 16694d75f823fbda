#!/usr/bin/env bash
# VM variant of run.sh: build the gfx950 kernels in-tree and serve the API on every interface.
set -euo pipefail
cd "$(dirname "$0")"
python setup.py build_ext
PENROZ_HOST="${PENROZ_HOST:-0.0.0.0}" exec python main.py

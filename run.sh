#!/usr/bin/env bash
# Build the gfx950 kernels in-tree (no-op when up to date) and start the API on 127.0.0.1:8000.
# Set PENROZ_HOST=0.0.0.0 to listen on every interface (VM use).
set -euo pipefail
cd "$(dirname "$0")"
python setup.py build_ext
exec python main.py

#!/bin/bash
# Builds a stand-alone probe executable from its .hip source next to it (gfx950), e.g.
#   tools/probes/build_probe.sh ipc_probe && tools/probes/ipc_probe
# Executables are build artefacts: git-ignored, rebuilt on demand.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
name="${1:?usage: build_probe.sh <probe name without .hip>}"
src="$here/$name.hip"
[ -f "$src" ] || { echo "no such probe source: $src" >&2; exit 1; }
if [ ! -x "$here/$name" ] || [ "$src" -nt "$here/$name" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -o "$here/$name" "$src"
fi
echo "$here/$name"

#!/bin/bash
# Build the Winograd tower probe (tools/winograd_probe.hip) and its
# attribution variants into tools/_build (build container; the .so files
# travel to the GPU box with the tree). Round 6, DESIGN.md §10.
set -eu
cd "$(dirname "$0")"
mkdir -p _build
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -shared -fPIC -std=c++17"
$H -DWP_Q=4 winograd_probe.hip -o _build/libwinoprobe_q4.so
$H -DWP_Q=8 winograd_probe.hip -o _build/libwinoprobe_q8.so
$H -DWP_Q=4 -DWP_SKIP_TRANSFORM winograd_probe.hip -o _build/libwinoprobe_noT.so
$H -DWP_Q=4 -DWP_SKIP_EPILOGUE winograd_probe.hip -o _build/libwinoprobe_noE.so
$H -DWP_Q=4 -DWP_SKIP_TRANSFORM -DWP_SKIP_EPILOGUE winograd_probe.hip -o _build/libwinoprobe_noTE.so

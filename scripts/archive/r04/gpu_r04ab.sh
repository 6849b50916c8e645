#!/usr/bin/env bash
# Round 4: pair-queue length against LDS occupancy. Modified Cornell's block (34 triangles)
# is 160 B over the 8-blocks-per-CU LDS share with 512-entry queues (7 blocks run), config 5's
# (depth 8: 7 path records per lane) fits 6; shorter queues (PT_PAIR_QUEUE) let 8 / 7 fit.
set -u
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
SKIP_TESTS=1 bash scripts/gpu_ab.sh \
  "m512::--scene mcornell --rough 0.3 --spp 1000" "m448:PT_PAIR_QUEUE=448:--scene mcornell --rough 0.3 --spp 1000" \
  "m384:PT_PAIR_QUEUE=384:--scene mcornell --rough 0.3 --spp 1000" "m512b::--scene mcornell --rough 0.3 --spp 1000" \
  "m448b:PT_PAIR_QUEUE=448:--scene mcornell --rough 0.3 --spp 1000" \
  "s512::--res 4096 --depth 8 --spp 64" "s288:PT_PAIR_QUEUE=288:--res 4096 --depth 8 --spp 64" \
  "s256:PT_PAIR_QUEUE=256:--res 4096 --depth 8 --spp 64" "s512b::--res 4096 --depth 8 --spp 64" "s288b:PT_PAIR_QUEUE=288:--res 4096 --depth 8 --spp 64" \
  "c512::--spp 1000" "c448:PT_PAIR_QUEUE=448:--spp 1000" \
  "m08_512::--scene mcornell --rough 0.8 --spp 1000" "m08_448:PT_PAIR_QUEUE=448:--scene mcornell --rough 0.8 --spp 1000"

# wide walk with the LDS freed by byte records: longer triangle queue, a partial third level in LDS
set -u
cd $GRAFT_REPO_ROOT
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh lds "s_base||$S" "s_q160|PT_WIDE_QUEUE_LEN=160|$S" "s_q192|PT_WIDE_QUEUE_LEN=192|$S" \
  "s_top3k|PT_WIDE_TOP_PARTIAL=1 PT_WIDE_TOP_BYTES=3072|$S" "s_top4k|PT_WIDE_TOP_PARTIAL=1 PT_WIDE_TOP_BYTES=4352|$S" \
  "s_base2||$S" "s_q160b|PT_WIDE_QUEUE_LEN=160|$S" "s_top4kb|PT_WIDE_TOP_PARTIAL=1 PT_WIDE_TOP_BYTES=4352|$S"

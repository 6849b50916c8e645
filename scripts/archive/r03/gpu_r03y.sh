# combinations: queue 160 with a partial third level (3 / 3.5 KiB of top nodes in LDS)
set -u
cd $GRAFT_REPO_ROOT
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh lds2 "s_base||$S" "s_q160_t3k|PT_WIDE_QUEUE_LEN=160 PT_WIDE_TOP_PARTIAL=1 PT_WIDE_TOP_BYTES=3072|$S" \
  "s_q160_t35|PT_WIDE_QUEUE_LEN=160 PT_WIDE_TOP_PARTIAL=1 PT_WIDE_TOP_BYTES=3584|$S" "s_t35|PT_WIDE_TOP_PARTIAL=1 PT_WIDE_TOP_BYTES=3584|$S" \
  "s_base2||$S" "s_q160_t3kb|PT_WIDE_QUEUE_LEN=160 PT_WIDE_TOP_PARTIAL=1 PT_WIDE_TOP_BYTES=3072|$S" "s_t3k|PT_WIDE_TOP_PARTIAL=1 PT_WIDE_TOP_BYTES=3072|$S"

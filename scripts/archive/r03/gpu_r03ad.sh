# re-tune at the final kernels: wide walk shade threshold, flat camera-regeneration threshold
set -u
cd $GRAFT_REPO_ROOT
S="--scene sphere --spp 1000"
STEPS=3 bash scripts/archive/r03/ab_r03.sh tune "s_t28||$S" "s_t24|PT_WIDE_THRESH=24|$S" "s_t32|PT_WIDE_THRESH=32|$S" "s_t36|PT_WIDE_THRESH=36|$S" "s_t28b||$S" \
  "c_r32||" "c_r24|PT_REGEN_THRESH=24|" "c_r40|PT_REGEN_THRESH=40|" "c_r32b||"

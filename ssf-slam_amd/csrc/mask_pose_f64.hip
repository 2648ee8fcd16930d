// mask_pose_f64.hip -- k_mask_pose on float64 pos / flow (ssf_mask_pose_batch_f64): the same
// kernel source as mask_pose.hip, instantiated for double storage in its own translation unit.
#define SSF_MASK_F64_TU 1
#include "mask_pose.hip"

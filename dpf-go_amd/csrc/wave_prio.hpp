// wave_prio.hpp — wave issue priority from progress feedback (device code),
// shared by the T-table tree kernel, the persistent batched-Eval kernel
// (dpf_kernels.hip) and the byte-sliced tree kernel (bs_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dpfk {

// Progress feedback (r06).  A kernel whose workgroup holds every wave of its
// CU keeps 16 LDS slots per SIMD (indexed by the hardware wave id, HW_ID
// bits [3:0]; SIMD in bits [5:4]; ~0 = empty or finished).  A wave stores its
// progress d in its slot, reads its SIMD's 16 slots and sets its issue
// priority by its lead over the slowest of them: 3 when it is the slowest,
// 2 within `near`, 1 within `far`, else 0.  Fixed progress thresholds cannot
// tell a wave that is ahead from one whose SIMD is simply fast.
__device__ __forceinline__ uint32_t* prog_slots(uint32_t* s_prog, uint32_t& slot) {
    const uint32_t hw = __builtin_amdgcn_s_getreg(0xF804);   // HW_ID
    slot = hw & 15u;
    return s_prog + 16 * ((hw >> 4) & 3u);
}
__device__ __forceinline__ void prio_by_lead(uint32_t* slots, uint32_t slot, uint32_t d, uint32_t near,
                                             uint32_t far) {
    slots[slot] = d;
    const uint4* q = reinterpret_cast<const uint4*>(slots);
    const uint4 a = q[0], b = q[1], e = q[2], f = q[3];
    uint32_t m = min(min(min(a.x, a.y), min(a.z, a.w)), min(min(b.x, b.y), min(b.z, b.w)));
    m = min(m, min(min(min(e.x, e.y), min(e.z, e.w)), min(min(f.x, f.y), min(f.z, f.w))));
    const uint32_t lead = d - __builtin_amdgcn_readfirstlane(m < d ? m : d);
    if (lead == 0) __builtin_amdgcn_s_setprio(3);
    else if (lead <= near) __builtin_amdgcn_s_setprio(2);
    else if (lead <= far) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

}  // namespace dpfk

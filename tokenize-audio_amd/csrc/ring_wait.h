// s_waitcnt vmcnt(n) with n folded to a constant by the caller's unrolled loop: the LDS-DMA ring waits of the fused
// q/k/v + attention kernel (qkv_attn.hip).  A ring wait counts only the DMA pieces certainly issued after the stage
// it waits for: the compiler keeps the DMA issues (inline asm with a memory clobber) in program order against the
// waits but moves the register-destined loads freely (it hoisted them above the wait of their step), so counting
// only what is certainly behind the stage is safe wherever those loads land; the compiler inserts their own waits.
#pragma once
#include "gemm_planes.h"

namespace mimi {

// (n > 31: waits for more than asked, vmcnt(31); n <= 0: everything)
__device__ __forceinline__ void vm_wait(int n) {
#define MIMI_VMW(c) \
    case c: asm volatile("s_waitcnt vmcnt(" #c ")" ::: "memory"); break;
    switch (n) {
        MIMI_VMW(1) MIMI_VMW(2) MIMI_VMW(3) MIMI_VMW(4) MIMI_VMW(5) MIMI_VMW(6) MIMI_VMW(7) MIMI_VMW(8)
        MIMI_VMW(9) MIMI_VMW(10) MIMI_VMW(11) MIMI_VMW(12) MIMI_VMW(13) MIMI_VMW(14) MIMI_VMW(15) MIMI_VMW(16)
        MIMI_VMW(17) MIMI_VMW(18) MIMI_VMW(19) MIMI_VMW(20) MIMI_VMW(21) MIMI_VMW(22) MIMI_VMW(23) MIMI_VMW(24)
        MIMI_VMW(25) MIMI_VMW(26) MIMI_VMW(27) MIMI_VMW(28) MIMI_VMW(29) MIMI_VMW(30) MIMI_VMW(31)
        default:
            if (n > 31)
                asm volatile("s_waitcnt vmcnt(31)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#undef MIMI_VMW
}

}  // namespace mimi

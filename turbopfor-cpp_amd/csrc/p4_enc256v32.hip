// p4_enc256v32.hip -- batch encode of 256v32 P4 blocks (p4Enc256v32 /
// p4D1Enc256v32, reference src/scalar/p4enc256v32_scalar.cpp:216-235 and
// p4d1enc256v32_scalar.cpp:7-15) on gfx950: the two-pass encoder of
// p4_enc256v32.h (plan -> run scan -> write).
//
// Only production kernels live in the library (the pass probes are in the
// measurement library, measure/tpf_measure.hip).  The single-pass designs
// measured against the two-pass encoder and rejected in round 2 (decoupled
// look-back over LDS-held tiles, the MALL-chunked pipelined launch, the
// persistent-grid form) were A/B'd from scripts/enc_variants.hip
// until round 4 (git history); round 5's slot encoder (values read once, a
// compaction pass) lost too and lives in the measurement library
// (measure/enc_slot.h).
#include "p4_enc256v32.h"

namespace tpf
{

size_t enc256v32_workspace(uint64_t nblocks) { return enc256::twopass_workspace(nblocks); }

hipError_t launch_enc256v32(const uint32_t * in, uint64_t nblocks, const uint32_t * starts, uint32_t start0, bool d1,
                            uint8_t * out, uint64_t out_cap, uint64_t * off, void * ws, size_t ws_bytes, hipStream_t stream)
{
    if (nblocks == 0)
        return fill_u32(off, 0u, 2, stream);
    if (nblocks + 1 > 0x7FFFFFFFull || ws_bytes < enc256v32_workspace(nblocks))
        return hipErrorInvalidValue;
    return enc256::launch_twopass<0, 0>(in, nblocks, starts, start0, d1, out, out_cap, off, ws, stream);
}

} // namespace tpf

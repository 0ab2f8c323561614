#pragma once
//
// turbopfor.h -- drop-in replacement for amosbird/TurboPFor-CPP's public header
// (reference include/turbopfor.h:1-82).  Every declaration below is
// signature-identical to the reference, C++ linkage, namespace turbopfor, so
// existing callers recompile and relink against libturbopfor_amd.so unchanged.
//
// Semantics follow the reference per call: encoders return one past the last
// byte written, decoders one past the last byte consumed; n == 0 returns the
// input pointer; the 128v/256v families always pack/unpack the layout's full
// 128/256 values (callers pass n equal to the block width).
//
// Execution: each call runs the MI355X (gfx950) HIP kernels of this library on
// the calling thread's device (one block = one launch through the batched
// C-ABI of turbopfor_gpu.h).  There is no CPU fallback: without a HIP device a
// call throws std::runtime_error.  For throughput use the batched entry points
// in turbopfor_gpu.h (device-resident) or turbopfor_capi.h (host streams).

#include <cstdint>

namespace turbopfor
{

// ---- 32-bit, horizontal layout, any n (reference turbopfor.h:9-18) ----------
unsigned char * p4Enc32(uint32_t * in, unsigned n, unsigned char * out);
unsigned char * p4D1Enc32(uint32_t * in, unsigned n, unsigned char * out, uint32_t start);
const unsigned char * p4Dec32(const unsigned char * in, unsigned n, uint32_t * out);
const unsigned char * p4D1Dec32(const unsigned char * in, unsigned n, uint32_t * out, uint32_t start);

// ---- 32-bit, 128-value 4-lane interleaved layout (reference :21-30) ---------
unsigned char * p4Enc128v32(uint32_t * in, unsigned n, unsigned char * out);
unsigned char * p4D1Enc128v32(uint32_t * in, unsigned n, unsigned char * out, uint32_t start);
const unsigned char * p4Dec128v32(const unsigned char * in, unsigned n, uint32_t * out);
const unsigned char * p4D1Dec128v32(const unsigned char * in, unsigned n, uint32_t * out, uint32_t start);

// ---- 32-bit, 256-value 8-lane interleaved layout (reference :33-42) ---------
unsigned char * p4Enc256v32(uint32_t * in, unsigned n, unsigned char * out);
unsigned char * p4D1Enc256v32(uint32_t * in, unsigned n, unsigned char * out, uint32_t start);
const unsigned char * p4Dec256v32(const unsigned char * in, unsigned n, uint32_t * out);
const unsigned char * p4D1Dec256v32(const unsigned char * in, unsigned n, uint32_t * out, uint32_t start);

// ---- 64-bit, horizontal layout, any n (reference :45-54) --------------------
unsigned char * p4Enc64(uint64_t * in, unsigned n, unsigned char * out);
unsigned char * p4D1Enc64(uint64_t * in, unsigned n, unsigned char * out, uint64_t start);
const unsigned char * p4Dec64(const unsigned char * in, unsigned n, uint64_t * out);
const unsigned char * p4D1Dec64(const unsigned char * in, unsigned n, uint64_t * out, uint64_t start);

// ---- 64-bit, 128-value hybrid layout (reference :57-67) ---------------------
unsigned char * p4Enc128v64(uint64_t * in, unsigned n, unsigned char * out);
unsigned char * p4D1Enc128v64(uint64_t * in, unsigned n, unsigned char * out, uint64_t start);
const unsigned char * p4Dec128v64(const unsigned char * in, unsigned n, uint64_t * out);
const unsigned char * p4D1Dec128v64(const unsigned char * in, unsigned n, uint64_t * out, uint64_t start);

// ---- 64-bit, 256 values = two 128v64 blocks (reference :69-80) --------------
unsigned char * p4Enc256v64(uint64_t * in, unsigned n, unsigned char * out);
unsigned char * p4D1Enc256v64(uint64_t * in, unsigned n, unsigned char * out, uint64_t start);
const unsigned char * p4Dec256v64(const unsigned char * in, unsigned n, uint64_t * out);
const unsigned char * p4D1Dec256v64(const unsigned char * in, unsigned n, uint64_t * out, uint64_t start);

} // namespace turbopfor

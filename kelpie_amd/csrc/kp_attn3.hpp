// kp_attn3.hpp -- kp_attn on bf16 MFMA with three-piece operands ("bf16x3").
//
// Same contract as kpattn::kp_attn (kp_attn.hpp): per query q over the frozen keys
// [key_begin, key_end) of its stream-K segment, the softmax statistics (m, l) and
// O = sum_e w(s_e) E_e with s_e = q . E_e, w = exp(s - m_ref) (ComplEx) or the
// BCE-through-sigmoid gradient (ConvE).  The contractions run on
// v_mfma_f32_16x16x32_bf16 (16x the per-clock rate of the f32-input MFMA on gfx950)
// with every fp32 operand x split exactly into three bf16 pieces
//   x = x0 + x1 + x2,  x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)
// (8 significant bits each: together the 24 of fp32).  A product a.b is taken as
//   a0 b0 + a0 b1 + a1 b0 + a0 b2 + a1 b1 + a2 b0      (six MFMAs)
// whose bf16 x bf16 products are exact in the fp32 accumulator; the dropped terms
// (a1 b2, a2 b1, a2 b2) are below 2^-24 of |a||b| (one fp32 rounding of the product;
// tests/test_bf16x3_split.py), so the scores and O agree with the fp32 path to fp32
// rounding (not bitwise: the accumulation order differs).  6 MFMAs of 16 cycles per 16x16x32 block against
// 8 f32 MFMAs of 32 cycles: 2.67x fewer MFMA cycles.
//
// Table image (built once per context, kp_split3_table): entity e is one ROW_B-byte
// row [piece 0: DP bf16 | piece 1 | piece 2 | pad], rows padded with zero rows to a
// multiple of 32, so a 32-entity key tile is TILE_B contiguous bytes and the LDS tile
// is the same bytes (one linear LDS-DMA copy).  The pad (split3_row_bytes) makes both
// the S-phase row reads and the O-phase transposed reads conflict-free (checked
// against the ds_read_b128 / ds_read_b64_tr_b16 lane groups of MI355X_MICROARCH §LDS:
// tools/attn3_banks.py); only the 16-deep tail reads stay 2-way.
//
// S phase (swapped, as kp_attn): S^T = E . Q^T, A = the entity rows (ds_read_b128 of
// 8 dims per lane), B = the query pieces held in VGPRs.  C row = entity 4g + r of a
// 16-entity sub-tile, C column = query c.
// O phase: O^T += E^T . P with the 32 entities of the tile as K.  k-slot j of lane
// group g is entity 4g + j (j < 4, sub-tile 0) or 16 + 4g + j - 4 (sub-tile 1): that
// is where the S^T accumulators already put P, so P's pieces are the B operand as
// they sit; A = E^T by two ds_read_b64_tr_b16 per piece (rows 4g.. and 16 + 4g..).
#pragma once
#include <type_traits>

#include "kp_attn.hpp"

#ifdef KP_ATTN3_STAMPS
#ifndef KP_DIAGNOSTIC_BUILD
#error "KP_ATTN3_STAMPS is a diagnostic build (make diag / tools/attn_micro.sh)"
#endif
// diagnostic: per-phase issue cycles of kp_attn3 summed over waves (s_memtime; its
// lgkmcnt return also perturbs the kernel's counted LDS waits, so this build's results
// are not checked): [S, softmax + split, O, tile end (DMA wait + barrier), tiles]
__device__ unsigned long long g_attn3_stamps[8];
#define KP3_STAMP(v) v = __builtin_amdgcn_s_memtime()
#define KP3_ACC(i, a, b) st_acc[i] += (b) - (a)
#else
#define KP3_STAMP(v) (void)0
#define KP3_ACC(i, a, b) (void)0
#endif

#ifdef KP_ATTN3_CLOCK
#ifndef KP_DIAGNOSTIC_BUILD
#error "KP_ATTN3_CLOCK is a diagnostic build (tools/attn_micro.sh)"
#endif
// diagnostic: the in-kernel clock (MI355X_MICROARCH 'DVFS give-back' item 6): thread 0 of
// each workgroup stamps s_memtime and s_memrealtime (100 MHz) when it starts and when it
// leaves; the stamps go only to this buffer, nothing else reads them
__device__ unsigned long long g_attn3_clock[4096][4];
#endif

#ifndef KP_O_AHEAD
#define KP_O_AHEAD 1
#endif
#ifndef KP_S_AHEAD
#define KP_S_AHEAD 1
#endif
static_assert(KP_S_AHEAD >= 1 && KP_S_AHEAD <= 2, "KP_S_AHEAD: 1..2 (lgkmcnt holds at most 15)");
// Diagnostic builds (timing only, wrong results): KP_DIAG_NO_S drops the S phase,
// KP_DIAG_NO_O the O phase, to see how the phases add up per tile.  They (and
// KP_ATTN_NODMA, KP_DIAG_DMA_LGKM0, KP_DMA_SPREAD_ALL) compile only together with
// KP_DIAGNOSTIC_BUILD, which `make diag` sets for the variants/ libraries; the product
// library can never carry one by a stray define.
#if (defined(KP_DIAG_NO_S) || defined(KP_DIAG_NO_O) || defined(KP_ATTN_NODMA) || defined(KP_DIAG_DMA_LGKM0) || \
     defined(KP_DMA_SPREAD_ALL) || defined(KP_DIAG_S4) || defined(KP_DIAG_DMA_VM0) || defined(KP_DIAG_M0SAVE) || defined(KP_DIAG_NO_OSTORE) || defined(KP_DIAG_EARLY_EXIT) || defined(KP_DIAG_O_HALF) || defined(KP_DIAG_S_HALF) || defined(KP_DIAG_XTILE_W)) && \
    !defined(KP_DIAGNOSTIC_BUILD)
#error "kp_attn3 diagnostic define without KP_DIAGNOSTIC_BUILD (these builds compute wrong results: make diag)"
#endif
// KP_DMA_SPREAD: the next tile's LDS-DMA goes out one piece per O block instead of one
// burst after the S phase, in the inline-asm read form (ASM) only: ComplEx D = 400
// 1.795 -> 1.713 ms (necessary) and 0.512 -> 0.492 ms (sufficient) per launch.  With
// the compiler-visible reads (ConvE D = 208) the spread form failed the GPU parity
// tests; that path keeps the burst until the cause is found.
#ifndef KP_DMA_SPREAD
#define KP_DMA_SPREAD 1
#endif
#ifndef KP_DMA_SPREAD_BCE
// the same choice for the ConvE (ATT_BCE_O) instantiation at two workgroups per CU: the
// burst (0) -- settled-clock micro, YAGO3-10 shape, interleaved: 1.816 / 1.823 ms against
// 1.830 / 1.838 (1, per O block), 1.847 / 1.850 (2), 1.829 / 1.836 (3, over the S steps)
#define KP_DMA_SPREAD_BCE 0
#endif
#ifndef KP_ILV
#define KP_ILV 1
#endif
#ifndef KP_DMA_GROUP
// buffer-descriptor LDS-DMA in groups of four consecutive pieces per wave: one M0 write and
// four buffer_load ... lds with offset:0/1024/2048/3072 in one asm statement (instead of an
// M0 write, an s_nop and one load per piece, each M0 write waiting on the previous load)
#define KP_DMA_GROUP 1
#endif
#ifndef KP_ATTN_PRIO
// wave issue priority of the attention waves (s_setprio) over the other batch's kernels'
// waves co-resident on their SIMDs (engine pipeline); 0 = the default priority
#define KP_ATTN_PRIO 0
#endif
#ifndef KP_ATTN_FULLTILE
#define KP_ATTN_FULLTILE 1  // full key tiles skip the per-key masks (bitwise the same)
#endif
#ifndef KP_ATTN_FULLTILE_ALL
#define KP_ATTN_FULLTILE_ALL 0  // ... on the compiler-visible read form (ConvE) as well
#endif
#ifndef KP_CV_EXACT_BCE
// ConvE BCE-through-sigmoid weight (kp_attn3 ATT_BCE_O and kp_conve.hip bce_g): bit 0 the
// accurate sigmoid (expf, IEEE division), bit 1 (p - y) * gs where p(1 - p) >= 1e-12 (the
// value the reference's ((p - y) / p(1 - p) * gs) * p(1 - p) rounds to in exact arithmetic)
#define KP_CV_EXACT_BCE 0
#endif
#ifndef KP_ASM_ALL
#define KP_ASM_ALL 0  // 1: the asm read form for every DB (ConvE included)
#endif
#ifndef KP_ASM_MIN_DB
// the asm read form from this width up (ConvE d = 200 is DB 13: asm since round 6, at two
// workgroups per CU; the compiler-visible form stays for the narrow test widths)
#define KP_ASM_MIN_DB 13
#endif
#ifndef KP_O_NT
#define KP_O_NT 0  // 1: nontemporal stores of the O partials (A/B)
#endif
#ifndef KP_O_SC1
#define KP_O_SC1 0  // 1: write-through (sc1) buffer stores of the O partials (A/B)
#endif
#ifndef KP_BUF_DMA
#define KP_BUF_DMA 1  // interleaved schedule: LDS-DMA by buffer_load ... lds with scalar offsets
#endif
#ifdef KP_DIAG_NO_O
#define KP_DIAG_O false
#else
#define KP_DIAG_O true
#endif
static_assert(KP_O_AHEAD >= 1 && KP_O_AHEAD <= 2, "KP_O_AHEAD: 1..2 (lgkmcnt holds at most 15)");

namespace kpattn {

constexpr float kPosInf = __builtin_huge_valf();

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

// bytes of one entity row of the split image and of a 32-entity tile
// (pad: 0 B for an odd number of 16-dim blocks, 32 B for an even one -- the padding
// that makes the S-phase ds_read_b128 and the O-phase ds_read_b64_tr_b16 conflict-free
// under gfx950's lane groups; a tile is then a whole number of KiB)
__host__ __device__ constexpr int split3_row_bytes(int DP) { return 3 * 2 * DP + ((DP / 16) % 2 ? 0 : 32); }
__host__ __device__ constexpr int split3_tile_bytes(int DP) { return 32 * split3_row_bytes(DP); }
// LDS-DMA pieces (1 KiB) per tile and the LDS bytes of kp_attn3 (two tile buffers)
__host__ __device__ constexpr int split3_pieces(int DP) { return (split3_tile_bytes(DP) + 1023) / 1024; }
// the asm read form (see lds_rd_bf8) and, with it, the interleaved schedule and the
// buffer-descriptor LDS-DMA (KP_BUF_DMA): every wave issues the same number of whole
// pieces, so a tile buffer is rounded up to a multiple of 4 pieces
__host__ __device__ constexpr bool attn3_asm(int DB) { return DB >= KP_ASM_MIN_DB || KP_ASM_ALL; }
__host__ __device__ constexpr bool attn3_bufdma(int DB) { return attn3_asm(DB) && KP_ILV && KP_BUF_DMA; }
__host__ __device__ constexpr int attn3_buf_pieces(int DB) {
  return attn3_bufdma(DB) ? (split3_pieces(16 * DB) + 3) / 4 * 4 : split3_pieces(16 * DB);
}
constexpr size_t attn3_lds_bytes(int DB) { return 2u * 1024u * (size_t)attn3_buf_pieces(DB); }

__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = __fsub_rn(x, (float)h);
  m = (__bf16)r1;
  const float r2 = __fsub_rn(r1, (float)m);
  l = (__bf16)r2;
}

// LDS operand reads, two forms (template flag ASM):
//  - compiler-visible loads: the compiler folds each read's constant offset into the
//    instruction and places counted lgkmcnt waits itself (best at two waves per SIMD:
//    ConvE d = 200, 2.80 -> 2.22 ms per launch);
//  - inline asm (ASM): the reads issue exactly one k-step / O block ahead with the
//    kernel's own counted waits, at the price of a v_add per read (best for the
//    register-bound one-wave-per-SIMD ComplEx d = 200 kernel: 0.383 vs 0.408 ms).
typedef __bf16 bf16v4 __attribute__((__vector_size__(8)));
// `off` is a compile-time constant after unrolling (< 64 KiB): the asm form carries it
// in the instruction's offset field, so a read costs no address arithmetic.
template <bool ASM>
__device__ __forceinline__ bf16x8 lds_rd_bf8(uint32_t addr, int off) {
  if constexpr (ASM) {
    bf16x8 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
    return v;
  } else {
    return *reinterpret_cast<const __attribute__((address_space(3))) bf16x8*>((uintptr_t)(addr + off));
  }
}
template <bool ASM>
__device__ __forceinline__ bf16x4 lds_rd_bf4(uint32_t addr, int off) {
  if constexpr (ASM) {
    bf16x4 v;
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
    return v;
  } else {
    return *reinterpret_cast<const __attribute__((address_space(3))) bf16x4*>((uintptr_t)(addr + off));
  }
}
template <bool ASM>
__device__ __forceinline__ bf16x4 lds_rd_tr(uint32_t addr, int off) {
  if constexpr (ASM) {
    bf16x4 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(off));
    return v;
  } else {
    const bf16v4 v = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
        reinterpret_cast<__attribute__((address_space(3))) bf16v4*>((uintptr_t)(addr + off)));
    return __builtin_bit_cast(bf16x4, v);
  }
}
template <bool ASM>
__device__ __forceinline__ bf16x8 tied3(bf16x8 v) {
  if constexpr (ASM) asm volatile("" : "+v"(v));
  return v;
}
template <bool ASM>
__device__ __forceinline__ bf16x4 tied3(bf16x4 v) {
  if constexpr (ASM) asm volatile("" : "+v"(v));
  return v;
}
template <bool ASM, int N>
__device__ __forceinline__ void lgkm_wait3() {
  if constexpr (ASM) lgkm_wait<N>();
}

// the six products of mfma3, in its order: piece of a, piece of b
constexpr int kPA[6] = {2, 1, 0, 1, 0, 0};
constexpr int kPB[6] = {0, 1, 2, 0, 1, 0};

// six-product a.b on one accumulator (smallest terms first)
__device__ __forceinline__ f32x4 mfma3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], c, 0, 0, 0);
  return c;
}
__device__ __forceinline__ f32x4 mfma3_k16(const bf16x4 (&a)[3], const bf16x4 (&b)[3], f32x4 c) {
#define KP_M16(x, y) \
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, x), __builtin_bit_cast(s16x4, y), c, 0, 0, 0)
  KP_M16(a[2], b[0]);
  KP_M16(a[1], b[1]);
  KP_M16(a[0], b[2]);
  KP_M16(a[1], b[0]);
  KP_M16(a[0], b[1]);
  KP_M16(a[0], b[0]);
#undef KP_M16
  return c;
}

// Split image of the fp32 table E [n_ent][DP]: one thread per (entity, 2 dims).
// The destination is zeroed by the caller (padding rows and bytes).
template <int DP>
__global__ void kp_split3_table(const float* __restrict__ E, int n_ent, uint8_t* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)n_ent * (DP / 2)) return;
  const int e = (int)(i / (DP / 2)), d = 2 * (int)(i % (DP / 2));
  __bf16 h[2], m[2], l[2];
  split3(E[(size_t)e * DP + d], h[0], m[0], l[0]);
  split3(E[(size_t)e * DP + d + 1], h[1], m[1], l[1]);
  __bf16* row = reinterpret_cast<__bf16*>(out + (size_t)e * split3_row_bytes(DP));
  row[d] = h[0];
  row[d + 1] = h[1];
  row[DP + d] = m[0];
  row[DP + d + 1] = m[1];
  row[2 * DP + d] = l[0];
  row[2 * DP + d + 1] = l[1];
}

// two workgroups per CU where the ConvE (BCE) form's two tile buffers fit twice in the LDS
// (ConvE d = 200: 229 registers); one otherwise (wider BCE forms would spill at 256)
template <int DB, int MODE>
constexpr int attn3_min_wgs() { return (MODE == ATT_BCE_O && 2 * attn3_lds_bytes(DB) <= 163840) ? 2 : 1; }

template <int DB, int MODE>
__global__ __launch_bounds__(256, (attn3_min_wgs<DB, MODE>())) void kp_attn3(const uint8_t* __restrict__ E3, int n_ent,
                                                   const float* __restrict__ Qpre, int nq, AttnWork wk,
                                                   float* __restrict__ out_m, float* __restrict__ out_l,
                                                   float* __restrict__ out_O, const float* __restrict__ qscale,
                                                   float ylo, const double* __restrict__ colpre) {
  constexpr bool WITH_O = MODE != ATT_SOFTMAX;
  constexpr int DP = 16 * DB;
  constexpr bool ASM = attn3_asm(DB);  // read form (see lds_rd_bf8)
  // interleaved schedule of the asm read form (KP_ILV, default on): reads two k-steps /
  // O blocks ahead, one per MFMA issue gap, order pinned by sched_barrier
  constexpr bool ILV = ASM && KP_ILV;
  constexpr int NK = DP / 32;         // full 32-deep k-steps of the S phase
  constexpr int TAIL = (DP % 32) / 16;  // one 16-deep k-step (16x16x16 MFMA) when DP % 32 == 16
  constexpr int KT = 32;
  constexpr int PART_B = 2 * DP;
  constexpr int ROW_B = split3_row_bytes(DP);
  constexpr bool BUFDMA = attn3_bufdma(DB);
  constexpr int PIECES = attn3_buf_pieces(DB);  // whole 1-KiB LDS-DMA pieces per tile buffer
  constexpr int BUF_B = 1024 * PIECES;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds3[];  // [2][BUF_B]

  const int tid = threadIdx.x;
#ifdef KP_DIAG_EARLY_EXIT
  // diagnostic: every workgroup leaves at once (same registers and LDS: the code below
  // stays reachable for a value the caller never passes), so a launch costs its dispatch
  if (ylo != 12345.f) return;
#endif
  if constexpr (KP_ATTN_PRIO > 0) __builtin_amdgcn_s_setprio(KP_ATTN_PRIO);
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, c = lane & 15;
  int key_begin = 0, key_end = 0;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint8_t*)lds3;
#ifdef KP_ATTN3_STAMPS
  unsigned long long st0 = 0, st1 = 0, st2 = 0, st3 = 0, st4 = 0;
  unsigned long long st_acc[5] = {0, 0, 0, 0, 0};
#endif

  // linear LDS-DMA of a tile: piece p = bytes [1024 p, 1024 p + 1024) of the tile,
  // wave w issues p = w, w + 4, ... (the image has >= 1 KiB of slack past its end)
  // buffer-descriptor form (BUFDMA): the descriptor covers the whole image (rows padded to
  // whole tiles plus 1 KiB of slack), the per-lane part is the constant voffset 16 lane and
  // everything that varies per piece is scalar (soffset, M0): no VALU per piece
  const __amdgpu_buffer_rsrc_t e3rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(E3), (short)0, (int)((n_ent + 31) / 32 * 32 * ROW_B + 1024), 0x00020000);
#if KP_O_SC1
  const __amdgpu_buffer_rsrc_t orsrc =
      __builtin_amdgcn_make_buffer_rsrc(out_O, (short)0, 0x7FFFFFFF, 0x00020000);
#endif
  auto bdma = [&](int tile, int buf, int p) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        e3rsrc, (__attribute__((address_space(3))) void*)(uintptr_t)(lds0 + (uint32_t)(buf * BUF_B + 1024 * p)), 16,
        16 * lane, (key_begin + tile * KT) * ROW_B + 1024 * p, 0, 0);
  };
  // KP_DMA_GROUP (BUFDMA): wave w issues the consecutive pieces w NPW .. w NPW + NPW - 1,
  // group g = pieces 4 g .. 4 g + 3 of them in one statement (the last group may be short)
  typedef int i32x4_t __attribute__((ext_vector_type(4)));
  const i32x4_t e3rs = {(int)(uint32_t)(uintptr_t)E3,
                        (int)(uint32_t)((uintptr_t)E3 >> 32) & 0xFFFF,
                        (int)((n_ent + 31) / 32 * 32 * ROW_B + 1024), 0x00020000};
  auto dma_group = [&](int tile, int buf, int g) {
    const int pb = w * ((PIECES + 3) / 4) + 4 * g;
    const uint32_t m0v = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds0 + (uint32_t)(buf * BUF_B + 1024 * pb)));
    const uint32_t so = (uint32_t)__builtin_amdgcn_readfirstlane((key_begin + tile * KT) * ROW_B + 1024 * pb);
    const int nleft = (PIECES + 3) / 4 - 4 * g;
    // M0 is reserved to the compiler (a clobber of it is not honoured): the group saves it
    // and puts it back, so a compiler-set M0 (the builtin LDS-DMA of bdma) stays valid
    uint32_t keep;
    if (nleft >= 4)
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen offset:1024 lds\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen offset:2048 lds\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen offset:3072 lds\n\ts_mov_b32 m0, %0" : "=&s"(keep) : "s"(m0v),
          "v"(16 * lane), "s"(e3rs), "s"(so)
          : "memory");
    else if (nleft == 3)
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen offset:1024 lds\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen offset:2048 lds\n\ts_mov_b32 m0, %0" : "=&s"(keep) : "s"(m0v),
          "v"(16 * lane), "s"(e3rs), "s"(so)
          : "memory");
    else if (nleft == 2)
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen offset:1024 lds\n\ts_mov_b32 m0, %0" : "=&s"(keep) : "s"(m0v),
          "v"(16 * lane), "s"(e3rs), "s"(so)
          : "memory");
    else if (nleft == 1)
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_nop 4\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
          "buffer_load_dwordx4 %2, %3, %4 offen lds\n\ts_mov_b32 m0, %0" : "=&s"(keep) : "s"(m0v),
          "v"(16 * lane), "s"(e3rs), "s"(so)
          : "memory");
  };
  constexpr bool DGROUP = KP_DMA_GROUP && BUFDMA;
  auto issue = [&](int tile, int buf) {
    const uint8_t* src = E3 + (size_t)(key_begin + tile * KT) * ROW_B + 16 * lane;
    if constexpr (KP_DMA_GROUP && BUFDMA) {
#pragma unroll
      for (int g = 0; g < ((PIECES + 3) / 4 + 3) / 4; ++g) dma_group(tile, buf, g);
      return;
    }
#pragma unroll
    for (int p0 = 0; p0 < PIECES; p0 += 4) {
      const int p = p0 + w;
      if constexpr (BUFDMA)
        bdma(tile, buf, p);
      else if (p < PIECES)
        glds16<ASM>(reinterpret_cast<const float*>(src + 1024 * p),
               __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(buf * BUF_B + 1024 * p)));
    }
  };
  // the wave's k-th piece of a tile's DMA (pieces w, w + 4, ...), for spreading the
  // copy over the O-phase MFMA stream (KP_DMA_SPREAD)
  constexpr int NPW = (PIECES + 3) / 4;
  constexpr int SPM = MODE == ATT_BCE_O ? KP_DMA_SPREAD_BCE : KP_DMA_SPREAD;  // spread mode of this instantiation
#ifdef KP_DMA_SPREAD_ALL
  constexpr bool SPREAD = SPM && WITH_O && KP_DIAG_O;  // diagnostic: every read form
#else
  constexpr bool SPREAD = SPM && ASM && WITH_O && KP_DIAG_O;
#endif
  // KP_DMA_SPREAD == 2 (interleaved schedule): the pieces go out evenly over the S steps
  // and the O blocks (slot k of NSLOT), so the copy's LDS writes share the LDS with the
  // lighter S-phase reads instead of piling onto the O phase's transposed reads
  // (== 3: over the S steps only)
  constexpr int NSLOT = (DP / 32 + (DP % 32) / 16) + (SPM == 3 ? 0 : DB);
  constexpr bool SPREAD2 = SPREAD && ILV && SPM >= 2;
  auto issue_piece = [&](int tile, int buf, int k) {
    const int p = 4 * k + w;
    if constexpr (BUFDMA)
      bdma(tile, buf, p);
    else if (p < PIECES)
      glds16<ASM>(reinterpret_cast<const float*>(E3 + (size_t)(key_begin + tile * KT) * ROW_B + 16 * lane + 1024 * p),
             __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(buf * BUF_B + 1024 * p)));
  };
  auto dma_slot = [&](int tile, int buf, int slot) {
#pragma unroll
    for (int k = 0; k < NPW; ++k)
      if ((k * NSLOT) / NPW == slot) issue_piece(tile, buf, k);
  };
#ifdef KP_ATTN3_CLOCK
  // stamped first thing (the asm's memory clobber keeps every load after it)
  unsigned long long ck_t0, ck_r0;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(ck_t0), "=s"(ck_r0)::"memory");
#endif
  const int QT = (nq + 63) / 64;
  // work segments: stream-K ranges (wk.ranges == 0) or XCD-grouped units (attn_plan_ranges)
  const long long total = (long long)QT * wk.ktq;
  long long it = wk.ranges ? 0 : (long long)blockIdx.x * wk.per_wg;
  const long long it_end = wk.ranges ? 0 : min(total, it + (long long)wk.per_wg);
  const int n_units = QT * wk.ranges;
  int unit = ((int)gridDim.x % 8 == 0) ? (int)(blockIdx.x % 8) * (int)(gridDim.x / 8) + (int)(blockIdx.x / 8)
                                       : (int)blockIdx.x;
  for (;;) {
    int qt, kt0, kt1, part;
    bool fill_rest;
    if (wk.ranges) {
      if (unit >= n_units) break;
      qt = unit % QT;
      part = unit / QT;
      kt0 = (int)((long long)part * wk.ktq / wk.ranges);
      kt1 = (int)((long long)(part + 1) * wk.ktq / wk.ranges);
      fill_rest = false;
      unit += (int)gridDim.x;
    } else {
      if (it >= it_end) break;
      qt = (int)(it / wk.ktq);
      kt0 = (int)(it - (long long)qt * wk.ktq);
      kt1 = (int)min((long long)wk.ktq, (long long)kt0 + (it_end - it));
      part = (int)blockIdx.x - (int)(((long long)qt * wk.ktq) / wk.per_wg);
      fill_rest = kt1 == wk.ktq;
      it += kt1 - kt0;
    }
    key_begin = kt0 * KT;
    key_end = min(n_ent, kt1 * KT);
    const int ntiles = kt1 - kt0;
    const int q = qt * 64 + 16 * w + c;
    const bool valid = q < nq;
    // ---- query pieces -> VGPRs: B operand of k-step s is q[32 s + 8 g + j]
    bf16x8 qb[NK > 0 ? NK : 1][3];
    bf16x4 qt4[3];
    float gsc = 0.f;
    if (MODE == ATT_BCE_O) gsc = valid ? qscale[q] : 0.f;
    {
      const float* qp = Qpre + (size_t)(valid ? q : 0) * DP;
#pragma unroll
      for (int s = 0; s < NK; ++s) {
        const float4 v0 = *reinterpret_cast<const float4*>(qp + 32 * s + 8 * g);
        const float4 v1 = *reinterpret_cast<const float4*>(qp + 32 * s + 8 * g + 4);
        const float f[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          __bf16 h, m, l;
          split3(valid ? f[j] : 0.f, h, m, l);
          qb[s][0][j] = h;
          qb[s][1][j] = m;
          qb[s][2][j] = l;
        }
      }
      if (TAIL) {
        const float4 v0 = *reinterpret_cast<const float4*>(qp + 32 * NK + 4 * g);
        const float f[4] = {v0.x, v0.y, v0.z, v0.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          __bf16 h, m, l;
          split3(valid ? f[j] : 0.f, h, m, l);
          qt4[0][j] = h;
          qt4[1][j] = m;
          qt4[2][j] = l;
        }
      }
    }
    f32x4 O[WITH_O ? DB : 1];
    float m_ref = kNegInf, l_run = 0.f;
    float csh = 0.f;  // the query's weight shift of this pass (centred accumulation, above)

    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int j = 0; j < (WITH_O ? DB : 1); ++j) O[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
      l_run = 0.f;
      float m_seen = kNegInf;
      if (ntiles > 0) issue(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#ifdef KP_DIAG_XTILE_W
      // diagnostic (wrong results, timing only): the upper bound of a cross-tile schedule.
      // The previous tile's softmax weights and P split are computed in pieces in the
      // S-phase MFMA gaps of this tile (as a schedule running S(t + 1) beside W(t) would),
      // and this tile's O phase uses them; the instruction mix per tile is the product's
      float scp[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      float pwn[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      float lacc = 0.f;
      bf16x8 pbn[3];
      // piece q of the previous tile's weights: 0..23 = value q / 3, step q % 3 (difference,
      // exp, centred sum); 24..47 = split of value (q - 24) / 3 into its three pieces
      float dtmp[8], htmp[8];
      auto wpiece = [&](int q) {
        if (q < 24) {
          const int j = q / 3, st = q % 3;
          if (st == 0) {
            dtmp[j] = scp[j >> 2][j & 3] - m_ref;
            m_seen = fmaxf(m_seen, scp[j >> 2][j & 3]);
          } else if (st == 1) {
            pwn[j] = __expf(dtmp[j]);
          } else {
            pwn[j] = __fsub_rn(pwn[j], csh);
            lacc += pwn[j];
          }
        } else if (q < 48) {
          const int j = (q - 24) / 3, st = (q - 24) % 3;
          if (st == 0) {
            const __bf16 h = (__bf16)pwn[j];
            pbn[0][j] = h;
            htmp[j] = __fsub_rn(pwn[j], (float)h);
          } else if (st == 1) {
            const __bf16 m = (__bf16)htmp[j];
            pbn[1][j] = m;
            htmp[j] = __fsub_rn(htmp[j], (float)m);
          } else {
            pbn[2][j] = (__bf16)htmp[j];
          }
        }
      };
#endif

      for (int t = 0; t < ntiles; ++t) {
        const int k0 = key_begin + t * KT;
        KP3_STAMP(st0);
        // next tile's DMA: with BUFDMA every tile issues it (the last one re-reads its own
        // rows into the idle buffer) so no piece sits behind a branch
        const bool dma_on = BUFDMA || t + 1 < ntiles;
        const int tn = t + 1 < ntiles ? t + 1 : t;
        const uint32_t tb = lds0 + (uint32_t)((t & 1) * BUF_B);
#if !defined(KP_ATTN_NODMA) && defined(KP_DMA_EARLY)
        // the other buffer was released by the previous tile's closing barrier
        if (t + 1 < ntiles) issue(t + 1, (t + 1) & 1);
#endif
        // ---- S^T per 16-entity sub-tile u (entity row 16u + c of the tile)
        // Both sub-tiles per k-step; each step's six operand reads are issued one step
        // ahead of its MFMAs (LDS returns in order: a counted lgkmcnt wait).
        f32x4 sc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
#ifdef KP_DIAG_S4
        f32x4 sc4[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
#endif
        const uint32_t rb = tb + (uint32_t)(c * ROW_B + 16 * g);
        const uint32_t rbt = rb - 8u * g;        // tail reads: 8 bytes per lane group
        constexpr uint32_t SUB_B = 16u * ROW_B;  // the second sub-tile's rows
        static_assert(SUB_B + 3 * PART_B + 64 * NK < 65536, "LDS read offsets exceed the 16-bit offset field");
        // k-step j < NK: six ds_read_b128 into buffer j % (SA + 1); step NK (TAIL): six
        // ds_read_b64.  Reads run KP_S_AHEAD steps ahead of their MFMAs.
        constexpr int SA = ILV ? 2 : KP_S_AHEAD;
        constexpr int LAST = NK + TAIL - 1;  // index of the last k-step
        bf16x8 ra[SA + 1][2][3];
        bf16x4 rt[2][3];
        auto load_full = [&](int s, int b) {
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int p = 0; p < 3; ++p) ra[b][u][p] = lds_rd_bf8<ASM>(rb, (int)(u * SUB_B) + p * PART_B + 64 * s);
        };
        auto load_tail = [&]() {
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int p = 0; p < 3; ++p)
              rt[u][p] = lds_rd_bf4<ASM>(rbt, (int)(u * SUB_B) + p * PART_B + 64 * NK);  // dims 32 NK + 4g ..
        };
        auto load_step = [&](int j) {
          if (j < NK)
            load_full(j, j % (SA + 1));
          else
            load_tail();
        };
#ifndef KP_DIAG_NO_S
        if constexpr (ILV) {
          // Interleaved form: step s's twelve MFMAs (the two sub-tiles' chains
          // alternating, each chain in mfma3's smallest-first order) carry step s + 2's
          // six reads in every other issue gap; sched_barrier pins that order, so the
          // reads never bunch up behind an MFMA group and a read has a whole step of
          // MFMAs (192 cycles) to land.  Before step s: wait until only step s + 1's
          // reads are pending.
          load_step(0);
          if (LAST >= 1) load_step(1);
#pragma unroll
          for (int s = 0; s <= LAST; ++s) {
            if (s < LAST)
              lgkm_wait<6>();
            else
              lgkm_wait<0>();
            __builtin_amdgcn_sched_barrier(0);
#if !defined(KP_ATTN_NODMA)
            if (SPREAD2 && dma_on) {
              dma_slot(tn, (t + 1) & 1, s);
              __builtin_amdgcn_sched_barrier(0);
            }
#endif
            const int b = s % 3;
#pragma unroll
            for (int k = 0; k < 6; ++k) {
#pragma unroll
              for (int u = 0; u < 2; ++u) {
#ifdef KP_DIAG_S4
                f32x4& acc = (s & 1) ? sc4[u] : sc[u];  // diagnostic: four accumulation chains
#else
                f32x4& acc = sc[u];
#endif
                if (s < NK)
                  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ra[b][u][kPA[k]], qb[s < NK ? s : 0][kPB[k]], acc, 0, 0,
                                                               0);
                else
                  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, rt[u][kPA[k]]),
                                                                  __builtin_bit_cast(s16x4, qt4[kPB[k]]), acc, 0, 0, 0);
#ifdef KP_DIAG_S_HALF
                if (u == 0 && s + 2 <= LAST && (k & 1) == 0) {  // diagnostic: half the S-phase operand reads
#else
                if (u == 0 && s + 2 <= LAST) {
#endif
                  // read k of step s + 2: (sub-tile k % 2, piece k / 2)
                  const int j = s + 2, uu = k & 1, pp = k >> 1;
                  if (j < NK)
                    ra[j % 3][uu][pp] = lds_rd_bf8<true>(rb, (int)(uu * SUB_B) + pp * PART_B + 64 * j);
                  else
                    rt[uu][pp] = lds_rd_bf4<true>(rbt, (int)(uu * SUB_B) + pp * PART_B + 64 * NK);
                }
#ifdef KP_DIAG_XTILE_W
                if (u == 1 && WITH_O) wpiece(6 * s + k);  // one piece per gap without a read
#endif
                __builtin_amdgcn_sched_barrier(0);
              }
            }
          }
#ifdef KP_DIAG_S4
          sc[0] += sc4[0];
          sc[1] += sc4[1];
#endif
        } else {
#pragma unroll
        for (int j = 0; j < SA && j <= LAST; ++j) load_step(j);
#pragma unroll
        for (int s = 0; s < NK; ++s) {
          // pending after step s's reads: steps s + 1 .. min(s + SA, LAST)
          if (s + SA <= LAST) {
            load_step(s + SA);
            lgkm_wait3<ASM, 6 * SA>();
          } else if (LAST - s >= 2) {
            lgkm_wait3<ASM, 12>();
          } else if (LAST - s == 1) {
            lgkm_wait3<ASM, 6>();
          } else {
            lgkm_wait3<ASM, 0>();
          }
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            bf16x8 a[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) a[p] = tied3<ASM>(ra[s % (SA + 1)][u][p]);
            sc[u] = mfma3(a, qb[s], sc[u]);
          }
        }
        if (TAIL) {
          lgkm_wait3<ASM, 0>();
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            bf16x4 a[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) a[p] = tied3<ASM>(rt[u][p]);
            sc[u] = mfma3_k16(a, qt4, sc[u]);
          }
        }
        }
#endif
#if !defined(KP_ATTN_NODMA) && !defined(KP_DMA_EARLY)
        // one burst here, or (KP_DMA_SPREAD, with an O phase) one piece per O block below:
        // a burst of ~19 LDS-DMA instructions per wave stalls the wave's issue behind the
        // texture-address queue before its O MFMAs start
        if (!SPREAD && t + 1 < ntiles) issue(t + 1, (t + 1) & 1);
#endif
        // O-phase operands: block m's six transposed reads (rows 4g.. and 16 + 4g.. of
        // each piece); lane c = 4 qq + pp reads row qq of the 4-row block, columns
        // 4 pp .. 4 pp + 3.  Block 0's are issued before the softmax, block m + 1's
        // before block m's MFMAs.
        const uint32_t ob = tb + (uint32_t)((4 * g + (c >> 2)) * ROW_B + 8 * (c & 3));
        // O-phase read-ahead depth: KP_O_AHEAD blocks (one block is 6 MFMAs = 96 cycles,
        // less than an LDS read's latency with four waves reading)
        constexpr int OA = ILV ? 2 : KP_O_AHEAD;
        bf16x4 ol[OA + 1][3], oh[OA + 1][3];
        auto load_o = [&](int m, int b) {
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            ol[b][p] = lds_rd_tr<ASM>(ob, p * PART_B + 32 * m);
            oh[b][p] = lds_rd_tr<ASM>(ob, 16 * ROW_B + p * PART_B + 32 * m);
          }
        };
        KP3_STAMP(st1);
        if (WITH_O && KP_DIAG_O) {
#pragma unroll
          for (int m = 0; m < OA && m < DB; ++m) load_o(m, m);
        }
        // weights of the tile (softmax or the BCE gradient) and the centred accumulation;
        // a full tile (every key < key_end: all but a range's last) runs without the key
        // masks (KP_ATTN_FULLTILE, the same bits)
        float pw[2][4];
        auto weights = [&](auto full_c) {
          constexpr bool FULL = decltype(full_c)::value;
          auto keep = [&](int u, int r) { return FULL || (k0 + 16 * u + 4 * g + r < key_end); };
        if (MODE == ATT_BCE_O) {
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#if KP_CV_EXACT_BCE & 1
              const float x0 = 1.0f / (1.0f + expf(-sc[u][r]));
#else
              const float x0 = __builtin_amdgcn_rcpf(1.0f + __expf(-sc[u][r]));
#endif
              const float w0 = (1.0f - x0) * x0;
#if KP_CV_EXACT_BCE & 2
              const float gw = w0 >= 1e-12f ? (x0 - ylo) * gsc
                                            : (((x0 - ylo) * __builtin_amdgcn_rcpf(1e-12f)) * gsc) * w0;
              pw[u][r] = keep(u, r) ? gw : 0.f;
#else
              pw[u][r] = keep(u, r) ? (((x0 - ylo) * __builtin_amdgcn_rcpf(fmaxf(w0, 1e-12f))) * gsc) * w0 : 0.f;
#endif
            }
        } else {
          float v[2][4];
          float tmax = kNegInf;
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[u][r] = keep(u, r) ? sc[u][r] : kNegInf;
              tmax = fmaxf(tmax, v[u][r]);
            }
          m_seen = fmaxf(m_seen, tmax);
          if (pass == 0 && t == 0) {
            float mq = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
            m_ref = fmaxf(mq, __shfl_xor(mq, 32, 64));
          }
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) pw[u][r] = __expf(v[u][r] - m_ref);
        }
        // centred accumulation: the first tile of a pass fixes the query's shift (the
        // smallest valid weight of that tile); every valid weight is accumulated minus it
        {
          if (t == 0) {
            float mn = kPosInf;
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (keep(u, r)) mn = fminf(mn, pw[u][r]);
            mn = fminf(mn, __shfl_xor(mn, 16, 64));
            mn = fminf(mn, __shfl_xor(mn, 32, 64));
            csh = (mn < kPosInf) ? mn : 0.f;
          }
          float lt = 0.f;
#pragma unroll
          for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int r = 0; r < 4; ++r) pw[u][r] = keep(u, r) ? __fsub_rn(pw[u][r], csh) : 0.f;
            lt += (pw[u][0] + pw[u][1]) + (pw[u][2] + pw[u][3]);
          }
          l_run += lt;
        }
        };
        // (the asm read form only: on the compiler-visible read form of the ConvE width the
        // same branch gave wrong, run-to-run different partials, with or without a
        // lgkmcnt(0) before each asm LDS-DMA piece -- DESIGN.md section 5)
#ifdef KP_DIAG_XTILE_W
        if (t == 0 || !ILV || !WITH_O)
#endif
        if (KP_ATTN_FULLTILE && (ASM || KP_ATTN_FULLTILE_ALL) && k0 + KT <= key_end)
          weights(std::true_type{});
        else
          weights(std::false_type{});
        if (WITH_O && KP_DIAG_O) {
          // P pieces in the B layout: element j of lane group g = entity 4g + j (j < 4)
          // or 16 + 4g + j - 4
          bf16x8 pb[3];
#ifdef KP_DIAG_XTILE_W
          if (ILV && t > 0) {
            pb[0] = pbn[0];
            pb[1] = pbn[1];
            pb[2] = pbn[2];
            l_run += lacc;
            lacc = 0.f;
          } else
#endif
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            __bf16 h, m, l;
            split3(pw[j >> 2][j & 3], h, m, l);
            pb[0][j] = h;
            pb[1][j] = m;
            pb[2][j] = l;
          }
#ifdef KP_DIAG_XTILE_W
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) scp[u][r] = sc[u][r];  // the next tile's gaps weight this tile
#endif
          KP3_STAMP(st2);
#pragma unroll
          for (int m = 0; m < DB; ++m) {
#if !defined(KP_ATTN_NODMA) && !defined(KP_DMA_EARLY)
            if (DGROUP && SPREAD && !SPREAD2 && dma_on) {
              if (m % 4 == 0 && m < NPW) dma_group(tn, (t + 1) & 1, m / 4);
              if (m == DB - 1)
                for (int g = (DB + 3) / 4; 4 * g < NPW; ++g) dma_group(tn, (t + 1) & 1, g);
            } else if (SPREAD && !SPREAD2 && dma_on) {
              if (m < NPW) {
                issue_piece(tn, (t + 1) & 1, m);
#ifdef KP_DIAG_DMA_LGKM0
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // diagnostic: drain after each piece
#endif
#ifdef KP_DIAG_DMA_VM0
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // diagnostic: each piece lands before what follows
#endif
              }
              if (m == DB - 1)
                for (int k = DB; k < NPW; ++k) issue_piece(tn, (t + 1) & 1, k);
            }
#endif
            if constexpr (ILV) {
              // block m + 2's six reads ride in block m's MFMA issue gaps (sched_barrier
              // pins the order); before block m only block m + 1's reads may be pending
              if (m + 1 < DB)
                lgkm_wait<6>();
              else
                lgkm_wait<0>();
              __builtin_amdgcn_sched_barrier(0);
#if !defined(KP_ATTN_NODMA)
              if (SPREAD2 && dma_on) {
                dma_slot(tn, (t + 1) & 1, NK + TAIL + m);
                __builtin_amdgcn_sched_barrier(0);
              }
#endif
              bf16x8 a[3];
#pragma unroll
              for (int p = 0; p < 3; ++p) {
                const bf16x4 x = ol[m % 3][p], y = oh[m % 3][p];
                a[p] = (bf16x8){x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
              }
#pragma unroll
              for (int k = 0; k < 6; ++k) {
                O[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[kPA[k]], pb[kPB[k]], O[m], 0, 0, 0);
#ifdef KP_DIAG_O_HALF
                if (m + 2 < DB && ((m + 2) & 1) == 0) {  // diagnostic: half the O-phase operand reads
#else
                if (m + 2 < DB) {
#endif
                  const int mm = m + 2, pp = k >> 1;
                  if (k & 1)
                    oh[mm % 3][pp] = lds_rd_tr<true>(ob, 16 * ROW_B + pp * PART_B + 32 * mm);
                  else
                    ol[mm % 3][pp] = lds_rd_tr<true>(ob, pp * PART_B + 32 * mm);
                }
                __builtin_amdgcn_sched_barrier(0);
              }
              continue;
            }
            // block m's reads are complete once at most (issued after them) reads are pending
            if (m + OA < DB) {
              load_o(m + OA, (m + OA) % (OA + 1));
              lgkm_wait3<ASM, 6 * OA>();
            } else if (DB - 1 - m >= 2) {
              lgkm_wait3<ASM, 12>();
            } else if (DB - 1 - m == 1) {
              lgkm_wait3<ASM, 6>();
            } else {
              lgkm_wait3<ASM, 0>();
            }
            bf16x8 a[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
              const bf16x4 x = tied3<ASM>(ol[m % (OA + 1)][p]), y = tied3<ASM>(oh[m % (OA + 1)][p]);
              a[p] = (bf16x8){x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
            }
            O[m] = mfma3(a, pb, O[m]);
          }
        }
        KP3_STAMP(st3);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        KP3_STAMP(st4);
        KP3_ACC(0, st0, st1);
        KP3_ACC(1, st1, st2);
        KP3_ACC(2, st2, st3);
        KP3_ACC(3, st3, st4);
#ifdef KP_ATTN3_STAMPS
        st_acc[4] += 1;
#endif
      }
      if (MODE == ATT_BCE_O) break;
      float mq = fmaxf(m_seen, __shfl_xor(m_seen, 16, 64));
      mq = fmaxf(mq, __shfl_xor(mq, 32, 64));
#if defined(KP_DIAG_NO_S) || defined(KP_DIAG_NO_O)
      break;
#endif
      if (pass == 1 || !__syncthreads_or(mq > m_ref + kMargin)) break;
      m_ref = mq;
    }

    float l_tot = l_run + __shfl_xor(l_run, 16, 64);
    l_tot += __shfl_xor(l_tot, 32, 64);
    if (ntiles > 0) {
      // the shifted-out part: csh * (number of keys) and csh * (sum of the keys' rows),
      // the latter from the fp64 prefix sums of the table over tiles
      l_tot = __fmaf_rn(csh, (float)(key_end - key_begin), l_tot);
      if (WITH_O) {
        const double* p0 = colpre + (size_t)kt0 * DP;
        const double* p1 = colpre + (size_t)kt1 * DP;
#pragma unroll
        for (int m = 0; m < DB; ++m) {
          const int d = 16 * m + 4 * g;  // 32-byte aligned quad of dims
          const double2 a0 = *reinterpret_cast<const double2*>(p0 + d), a1 = *reinterpret_cast<const double2*>(p0 + d + 2);
          const double2 b0 = *reinterpret_cast<const double2*>(p1 + d), b1 = *reinterpret_cast<const double2*>(p1 + d + 2);
          O[m][0] = __fmaf_rn(csh, (float)(b0.x - a0.x), O[m][0]);
          O[m][1] = __fmaf_rn(csh, (float)(b0.y - a0.y), O[m][1]);
          O[m][2] = __fmaf_rn(csh, (float)(b1.x - a1.x), O[m][2]);
          O[m][3] = __fmaf_rn(csh, (float)(b1.y - a1.y), O[m][3]);
        }
      }
    }
    if (valid) {
      const size_t o = (size_t)part * nq + q;
      if (g == 0 && MODE != ATT_BCE_O) {
        out_m[o] = m_ref;
        out_l[o] = l_tot;
      }
#ifdef KP_DIAG_NO_OSTORE
      if (false) {  // diagnostic: the O partials are not written (wrong results)
#else
      if (WITH_O) {
#endif
        // O^T block m: lane (g, c) holds dims 16 m + 4 g + r of query c
        float* dst = out_O + o * DP;
#pragma unroll
        for (int m = 0; m < DB; ++m) {
#if KP_O_SC1
          // write-through (sc1): the lines leave L2 as they are written instead of at the
          // kernel's end (the partials are read once, by the next kernel, on any XCD)
          typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, O[m]), orsrc,
                                                 (int)((o * DP + 16 * m + 4 * g) * sizeof(float)), 0, 16);
#elif KP_O_NT
          // streamed past L2: the partials are read once, by the next kernel
          __builtin_nontemporal_store(O[m], reinterpret_cast<f32x4*>(dst + 16 * m + 4 * g));
#else
          *reinterpret_cast<float4*>(dst + 16 * m + 4 * g) = make_float4(O[m][0], O[m][1], O[m][2], O[m][3]);
#endif
        }
      }
    }
    if (fill_rest && valid) {
      for (int pp = part + 1; pp < wk.n_parts; ++pp) {
        const size_t o = (size_t)pp * nq + q;
        if (g == 0 && MODE != ATT_BCE_O) {
          out_m[o] = kNegInf;
          out_l[o] = 0.f;
        }
        if (WITH_O) {
          float* dst = out_O + o * DP;
          for (int d = 4 * g; d < DP; d += 16) *reinterpret_cast<float4*>(dst + d) = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
  }
#ifdef KP_ATTN3_STAMPS
  if (lane == 0)
    for (int i = 0; i < 5; ++i) atomicAdd(&g_attn3_stamps[i], st_acc[i]);
#endif
#ifdef KP_ATTN3_CLOCK
  {
    // stamped last, after this wave's stores have completed
    unsigned long long ck_t1, ck_r1;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)"
                 : "=s"(ck_t1), "=s"(ck_r1)::"memory");
    if (tid == 0 && blockIdx.x < 4096) {
      g_attn3_clock[blockIdx.x][0] = ck_t0;
      g_attn3_clock[blockIdx.x][1] = ck_r0;
      g_attn3_clock[blockIdx.x][2] = ck_t1;
      g_attn3_clock[blockIdx.x][3] = ck_r1;
    }
  }
#endif
}

// Host: the split image of c->dE (row stride DP = c->dp), built once per context.
template <int DB>
const uint8_t* split3_image(kp_ctx* c) {
  constexpr int DP = 16 * DB;
  KP_REQUIRE(c->dp == DP, "attn3: table stride mismatch");
  if (!c->e3_ready) {
    const size_t n_pad = (size_t)(c->n_ent + 31) / 32 * 32;
    const size_t bytes = n_pad * split3_row_bytes(DP) + 1024;  // slack for the last tile's whole DMA pieces
    uint8_t* d = reinterpret_cast<uint8_t*>(c->e3.ensure(bytes));
    KP_HIP(hipMemsetAsync(d, 0, bytes, c->stream));
    const long long n = (long long)c->n_ent * (DP / 2);
    hipLaunchKernelGGL((kp_split3_table<DP>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, c->stream, c->dE,
                       c->n_ent, d);
    KP_HIP(hipGetLastError());
    c->e3_ready = true;
  }
  return c->e3.as<uint8_t>();
}

// Prefix sums of the fp32 table over 32-entity tiles, in fp64: colpre[t][d] = sum of
// E[e][d] over e < min(32 t, n_ent).  Tile sums first (one thread per (tile, dim)), then
// one thread per dim scans the tiles.
template <int DP>
__global__ void kp_tile_sums(const float* __restrict__ E, int n_ent, double* __restrict__ ts) {
  const int t = blockIdx.x, d = threadIdx.x;
  if (d >= DP) return;
  double s = 0.0;
  const int e1 = min(n_ent, 32 * t + 32);
  for (int e = 32 * t; e < e1; ++e) s += (double)E[(size_t)e * DP + d];
  ts[(size_t)t * DP + d] = s;
}
template <int DP>
__global__ void kp_tile_prefix(const double* __restrict__ ts, int ntiles, double* __restrict__ pre) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= DP) return;
  double s = 0.0;
  pre[d] = 0.0;
  for (int t = 0; t < ntiles; ++t) {
    s += ts[(size_t)t * DP + d];
    pre[(size_t)(t + 1) * DP + d] = s;
  }
}
template <int DB>
const double* tile_prefix(kp_ctx* c) {
  constexpr int DP = 16 * DB;
  if (!c->e3pre_ready) {
    const int ntiles = (c->n_ent + 31) / 32;
    double* ts = reinterpret_cast<double*>(c->e3ts.ensure(sizeof(double) * (size_t)ntiles * DP));
    double* pre = reinterpret_cast<double*>(c->e3pre.ensure(sizeof(double) * (size_t)(ntiles + 1) * DP));
    hipLaunchKernelGGL((kp_tile_sums<DP>), dim3((unsigned)ntiles), dim3((DP + 63) / 64 * 64), 0, c->stream, c->dE,
                       c->n_ent, ts);
    KP_HIP(hipGetLastError());
    hipLaunchKernelGGL((kp_tile_prefix<DP>), dim3((DP + 63) / 64), dim3(64), 0, c->stream, ts, ntiles, pre);
    KP_HIP(hipGetLastError());
    c->e3pre_ready = true;
  }
  return c->e3pre.as<double>();
}

// Host: co-resident kp_attn3 workgroups per CU (registers and LDS) of the instantiation a
// caller launches (MODE: ATT_SOFTMAX_O for ComplEx, whose ATT_SOFTMAX launch is no larger;
// ATT_BCE_O for ConvE), cached per context and mode.  Taking the smaller of the two modes
// for both cost ConvE its second workgroup per CU once its read form was the asm one
// (kp_attn3<13, ATT_SOFTMAX_O> holds 316 registers there, kp_attn3<13, ATT_BCE_O> 232).
template <int DB, int MODE = ATT_SOFTMAX_O>
int attn3_wpc(kp_ctx* c) {
  static_assert(MODE == ATT_SOFTMAX_O || MODE == ATT_BCE_O, "attn3_wpc: the launched O mode");
  int& slot = c->attn3_wpc[MODE == ATT_BCE_O ? 1 : 0];
  if (slot <= 0) {
    int n = 0;
    KP_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kp_attn3<DB, MODE>, 256, attn3_lds_bytes(DB)));
    slot = std::max(1, n);
  }
  return slot;
}

// Host: the partition of the context's attention kernel.  kp_attn3 takes the XCD-grouped
// aligned ranges unless their quantisation costs more than 40 % over stream-K's
// balanced split: the L2 reuse they buy (FETCH_SIZE 14x lower, L2 hit rate 2 -> 91 %)
// outweighs a worse balance.  KP_ATTN_PART=streamk
// forces stream-K, KP_ATTN_PART=ranges the ranges (parity tests run both).  The fp32
// kp_attn always uses stream-K.
inline AttnPlan attn_plan_ctx(const kp_ctx* c, int nq, int n_ent, int slots) {
  const AttnPlan sk = attn_plan(nq, n_ent, slots);
  if (c->attn_mode != 1 || c->attn_part == 1) return sk;
  const AttnPlan r = attn_plan_ranges(nq, n_ent, slots);
  if (c->attn_part == 2) return r;
  const long long QT = (nq + 63) / 64, S = r.wk.ranges, ktq = r.wk.ktq;
  const long long n_wg = std::max(8, slots / 8 * 8);
  const long long cost_r = (QT * S + n_wg - 1) / n_wg * ((ktq + S - 1) / S + 2);
  const long long cost_sk = (long long)sk.wk.per_wg + 2;
  // measured on the interleaved kernel (tools/attn_micro.hip, FB15k-237 ComplEx, nq 800 -
  // 5,000): the ranges ran 9-21 % faster than stream-K at every size although their
  // quantisation was up to 25 % worse (profiles/r02o_attn_partition.jsonl)
  (void)n_ent;
  return 100 * cost_r <= 140 * cost_sk ? r : sk;
}

template <int DB, int MODE>
void launch_attn3(kp_ctx* c, int n_ent, const float* Q, int nq, const AttnPlan& plan, float* m, float* l, float* O,
                  const float* qscale, float ylo) {
  KP_REQUIRE(n_ent == c->n_ent, "attn3: key count differs from the table's (tile prefix sums)");
  // the buffer descriptor's record count and the per-piece soffset are 32-bit: the split
  // image (ROW_B per entity, whole tiles, 1 KiB slack) must stay below 2^31 bytes
  // (D = 400: ~890k entities; out-of-range buffer loads would return zeros silently)
  KP_REQUIRE((long long)(n_ent + 31) / 32 * 32 * split3_row_bytes(16 * DB) + 1024 < (1LL << 31),
             "attn3: table too large for the 32-bit buffer descriptor of the split image");
  const uint8_t* E3 = split3_image<DB>(c);
  const double* pre = tile_prefix<DB>(c);
  hipLaunchKernelGGL((kp_attn3<DB, MODE>), dim3(plan.n_wg), dim3(256), attn3_lds_bytes(DB), c->stream, E3, n_ent, Q,
                     nq, plan.wk, m, l, O, qscale, ylo, pre);
  KP_HIP(hipGetLastError());
}

}  // namespace kpattn

// Lane-vector layer of the wave-cooperative latency engine ("wv"): one wave per item, one 25-bit
// limb per lane (wfield.h), so a single verification uses all 64 lanes instead of one.
//
// Device build: a lane vector V is the lane's own uint32_t and every operation below compiles to one
// or two VALU / DPP / ds instructions. Host build (-DWV_HOST, tools/wvtest.cpp): V is a struct of 64
// lanes and the same operations are emulated lane by lane with the mappings tools/dpp_probe.hip
// checked on the MI355X (profiles/r03_dpp_probe.txt), so the whole engine runs on the CPU against the
// oracle before it runs on the GPU.
//
// Lane layout: lane l, row r = l / 16 (DPP rows of 16 lanes), half h = l / 32. A field value occupies
// the even row of its half (lanes 32h .. 32h + 15); the odd row is the product's high workspace and
// is zero in a stored value ("value form").
#pragma once
#include <stdint.h>
#include <type_traits>
#include <utility>

#ifdef WV_HOST
#include <string.h>
#define WVI inline
namespace wv {
struct V {
  uint32_t v[64];
};
struct V64 {
  uint64_t v[64];
};
struct M {
  bool v[64];
};
#define WV_LANES for (int l = 0; l < 64; l++)
WVI V vsplat(uint32_t s) {
  V r;
  WV_LANES r.v[l] = s;
  return r;
}
WVI V64 vsplat64(uint64_t s) {
  V64 r;
  WV_LANES r.v[l] = s;
  return r;
}
#define WV_BIN(op)                                        \
  WVI V operator op(const V& a, const V& b) {             \
    V r;                                                  \
    WV_LANES r.v[l] = a.v[l] op b.v[l];                   \
    return r;                                             \
  }                                                       \
  WVI V operator op(const V& a, uint32_t b) {             \
    V r;                                                  \
    WV_LANES r.v[l] = a.v[l] op b;                        \
    return r;                                             \
  }                                                       \
  WVI V operator op(uint32_t a, const V& b) {             \
    V r;                                                  \
    WV_LANES r.v[l] = a op b.v[l];                        \
    return r;                                             \
  }
WV_BIN(+)
WV_BIN(-)
WV_BIN(*)
WV_BIN(&)
WV_BIN(|)
WV_BIN(^)
WV_BIN(>>)
WV_BIN(<<)
#undef WV_BIN
#define WV_CMP(op)                                        \
  WVI M operator op(const V& a, const V& b) {             \
    M r;                                                  \
    WV_LANES r.v[l] = a.v[l] op b.v[l];                   \
    return r;                                             \
  }                                                       \
  WVI M operator op(const V& a, uint32_t b) {             \
    M r;                                                  \
    WV_LANES r.v[l] = a.v[l] op b;                        \
    return r;                                             \
  }
WV_CMP(==)
WV_CMP(!=)
WV_CMP(<)
WV_CMP(>)
WV_CMP(>=)
WV_CMP(<=)
#undef WV_CMP
WVI M operator&(const M& a, const M& b) {
  M r;
  WV_LANES r.v[l] = a.v[l] && b.v[l];
  return r;
}
WVI M operator|(const M& a, const M& b) {
  M r;
  WV_LANES r.v[l] = a.v[l] || b.v[l];
  return r;
}
WVI M operator!(const M& a) {
  M r;
  WV_LANES r.v[l] = !a.v[l];
  return r;
}
WVI V sel(const M& c, const V& a, const V& b) {
  V r;
  WV_LANES r.v[l] = c.v[l] ? a.v[l] : b.v[l];
  return r;
}
WVI V lane_id() {
  V r;
  WV_LANES r.v[l] = (uint32_t)l;
  return r;
}
// acc + a * b (v_mad_u64_u32)
WVI V64 mad(const V& a, const V& b, const V64& acc) {
  V64 r;
  WV_LANES r.v[l] = acc.v[l] + (uint64_t)a.v[l] * b.v[l];
  return r;
}
WVI V64 mad(const V& a, uint32_t b, const V64& acc) {
  V64 r;
  WV_LANES r.v[l] = acc.v[l] + (uint64_t)a.v[l] * b;
  return r;
}
WVI V64 operator>>(const V64& a, int s) {
  V64 r;
  WV_LANES r.v[l] = a.v[l] >> s;
  return r;
}
// acc + (int32)a * (int32)b, two's complement (v_mad_i64_i32)
WVI V64 smad(const V& a, const V& b, const V64& acc) {
  V64 r;
  WV_LANES r.v[l] = acc.v[l] + (uint64_t)((int64_t)(int32_t)a.v[l] * (int64_t)(int32_t)b.v[l]);
  return r;
}
// arithmetic shift of the two's-complement value
WVI V64 sar64(const V64& a, int s) {
  V64 r;
  WV_LANES r.v[l] = (uint64_t)((int64_t)a.v[l] >> s);
  return r;
}
WVI V sar32(const V& a, int s) {
  V r;
  WV_LANES r.v[l] = (uint32_t)((int32_t)a.v[l] >> s);
  return r;
}
WVI V64 widen(const V& a) {
  V64 r;
  WV_LANES r.v[l] = a.v[l];
  return r;
}
WVI V64 add64(const V64& a, const V64& b) {
  V64 r;
  WV_LANES r.v[l] = a.v[l] + b.v[l];
  return r;
}
WVI V lo32(const V64& a) {
  V r;
  WV_LANES r.v[l] = (uint32_t)a.v[l];
  return r;
}
WVI V hi32(const V64& a) {
  V r;
  WV_LANES r.v[l] = (uint32_t)(a.v[l] >> 32);
  return r;
}
// (uint32)(a >> s), s < 32: v_alignbit on the two halves
WVI V shr64_lo(const V64& a, int s) {
  V r;
  WV_LANES r.v[l] = (uint32_t)(a.v[l] >> s);
  return r;
}
WVI V64 join64(const V& lo, const V& hi) {
  V64 r;
  WV_LANES r.v[l] = ((uint64_t)hi.v[l] << 32) | lo.v[l];
  return r;
}
// ---- cross-lane (DPP / permlane); bound_ctrl: lanes without a source read 0
template <int j>
WVI V row_shr(const V& x) {  // lane l <- l - j within the row
  V r;
  WV_LANES r.v[l] = (l % 16) >= j ? x.v[l - j] : 0u;
  return r;
}
template <int j>
WVI V row_shl(const V& x) {  // lane l <- l + j within the row
  V r;
  WV_LANES r.v[l] = (l % 16) + j < 16 ? x.v[l + j] : 0u;
  return r;
}
WVI V wave_shr1(const V& x) {  // lane l <- l - 1 across the wave
  V r;
  WV_LANES r.v[l] = l ? x.v[l - 1] : 0u;
  return r;
}
template <int i>
WVI V row_bcast(const V& x) {  // row_newbcast:i: lane l <- lane 16 (l / 16) + i
  V r;
  WV_LANES r.v[l] = x.v[16 * (l / 16) + i];
  return r;
}
// v_permlane16_swap(x, y): .a = x with its odd rows <- y's even rows; .b = y with its even rows <- x's odd rows
struct VP {
  V a, b;
};
WVI VP pl16_swap(const V& x, const V& y) {
  VP r;
  WV_LANES {
    const int row = l / 16;
    r.a.v[l] = (row & 1) ? y.v[l - 16] : x.v[l];
    r.b.v[l] = (row & 1) ? y.v[l] : x.v[l + 16];
  }
  return r;
}
// v_permlane32_swap(x, y): .a = [x.h0 | y.h0], .b = [x.h1 | y.h1]
WVI VP pl32_swap(const V& x, const V& y) {
  VP r;
  WV_LANES {
    r.a.v[l] = l >= 32 ? y.v[l - 32] : x.v[l];
    r.b.v[l] = l >= 32 ? y.v[l] : x.v[l + 32];
  }
  return r;
}
WVI uint64_t ballot(const M& m) {
  uint64_t b = 0;
  WV_LANES b |= (uint64_t)m.v[l] << l;
  return b;
}
WVI uint32_t lane_val(const V& x, int l) { return x.v[l]; }  // v_readlane
// ---- LDS: base = this wave's region, per-lane word offsets
WVI V lds_ld(const uint32_t* base, const V& off) {
  V r;
  WV_LANES r.v[l] = base[off.v[l]];
  return r;
}
WVI void lds_st(uint32_t* base, const V& off, const V& x) { WV_LANES base[off.v[l]] = x.v[l]; }
// global / constant table loads, per-lane index
WVI V gld(const uint32_t* base, const V& idx) { return lds_ld(base, idx); }
WVI void gst(uint32_t* base, const V& idx, const V& x) { lds_st(base, idx, x); }
#undef WV_LANES
}  // namespace wv

#else  // device
#include <hip/hip_runtime.h>
#define WVI __device__ __forceinline__
namespace wv {
typedef uint32_t V;
typedef uint64_t V64;
typedef bool M;
WVI V vsplat(uint32_t s) { return s; }
WVI V64 vsplat64(uint64_t s) { return s; }
WVI V sel(M c, V a, V b) { return c ? a : b; }
WVI V lane_id() { return __lane_id(); }
WVI V64 mad(V a, V b, V64 acc) { return acc + (uint64_t)a * b; }
WVI V64 smad(V a, V b, V64 acc) { return acc + (uint64_t)((int64_t)(int32_t)a * (int64_t)(int32_t)b); }
WVI V64 sar64(V64 a, int s) { return (uint64_t)((int64_t)a >> s); }
WVI V sar32(V a, int s) { return (uint32_t)((int32_t)a >> s); }
WVI V64 widen(V a) { return a; }
WVI V64 add64(V64 a, V64 b) { return a + b; }
WVI V lo32(V64 a) { return (uint32_t)a; }
WVI V hi32(V64 a) { return (uint32_t)(a >> 32); }
WVI V shr64_lo(V64 a, int s) { return (uint32_t)(a >> s); }
WVI V64 join64(V lo, V hi) { return ((uint64_t)hi << 32) | lo; }
// DPP controls: row_shl:j = 0x100+j, row_shr:j = 0x110+j, wave_shr:1 = 0x138, row_newbcast:i = 0x150+i
#define WV_DPP(x, ctrl) ((uint32_t)__builtin_amdgcn_update_dpp(0, (int)(x), (ctrl), 0xf, 0xf, true))
template <int j>
WVI V row_shr(V x) {
  if constexpr (j == 0)
    return x;
  else
    return WV_DPP(x, 0x110 + j);
}
template <int j>
WVI V row_shl(V x) {
  if constexpr (j == 0)
    return x;
  else
    return WV_DPP(x, 0x100 + j);
}
template <int i>
WVI V row_bcast(V x) {
  // every lane is written (all rows and banks, an in-row source), so no "old" value: mov_dpp leaves it
  // undefined and the compiler does not zero the destination first
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x150 + i, 0xf, 0xf, false);
}
WVI V wave_shr1(V x) { return WV_DPP(x, 0x138); }
struct VP {
  V a, b;
};
WVI VP pl16_swap(V x, V y) {
  auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  return {(V)r[0], (V)r[1]};
}
WVI VP pl32_swap(V x, V y) {
  auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  return {(V)r[0], (V)r[1]};
}
WVI uint64_t ballot(M m) { return __builtin_amdgcn_ballot_w64(m); }
WVI uint32_t lane_val(V x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
WVI V lds_ld(const uint32_t* base, V off) { return base[off]; }
WVI void lds_st(uint32_t* base, V off, V x) { base[off] = x; }
WVI V gld(const uint32_t* base, V idx) { return base[idx]; }
WVI void gst(uint32_t* base, V idx, V x) { base[idx] = x; }
}  // namespace wv
#endif

namespace wv {
// compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1 (DPP controls are immediates)
template <typename F, int... I>
WVI void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
WVI void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}
}  // namespace wv

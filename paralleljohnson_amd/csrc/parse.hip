// parse.hip — SNAP edge-list text -> COO on the GPU (read_webgraph,
// ParallelJohnson.cpp:66-105).
//
// The text is split into 64-byte segments, one per lane (16 KiB per 256-thread
// block). Pass 1 counts, per block, the line starts whose first byte is a
// decimal digit (the reference's edge test :73/:91); an exclusive scan turns
// the counts into edge indices, so edges keep file order. Pass 2 recomputes
// the per-lane line-start bitmask and parses each of its lines with
// `istringstream >> int >> int` semantics (:92-93): leading blanks skipped,
// optional sign, digits; a non-numeric field reads as 0; extra columns are
// ignored. Lines the reference turns into undefined behaviour (second field
// missing, negative id, id overflow) are reported by byte offset.
#include <chrono>

#include "devutil.h"

namespace pj {

namespace {

constexpr int PB = 256;
constexpr int PSEG = 64;
constexpr i64 PCHUNK = (i64)PB * PSEG;
constexpr i64 PTAIL = 512;  // bytes past the chunk staged with it (lines crossing the chunk end)
constexpr i64 ID_LIMIT = 2147483646;  // N = max + 1 must fit the reference's int (:319)

__device__ __forceinline__ bool is_digit(u32 c) { return (c - (u32)'0') < 10u; }
__device__ __forceinline__ bool is_blank(u32 c) {
    return c == ' ' || c == '\t' || c == '\v' || c == '\f' || c == '\r';
}

// Bitmask of positions p in [seg, seg+64) with text[p] a digit and
// (p == 0 or text[p-1] == '\n'). The buffer is zero-padded to a multiple of
// 64 bytes (+PTAIL), and '\0' is neither a digit nor a newline. `prev` is
// text[seg - 1] ('\n' at seg 0).
__device__ __forceinline__ u64 line_start_mask_w(const u32 (&words)[16], u32 prev) {
    u64 mask = 0;
#pragma unroll
    for (int k = 0; k < 64; ++k) {
        const u32 c = (words[k >> 2] >> ((k & 3) * 8)) & 0xFFu;
        if (prev == (u32)'\n' && is_digit(c)) mask |= 1ull << k;
        prev = c;
    }
    return mask;
}
__device__ __forceinline__ u64 line_start_mask(const uint4* __restrict__ p4, u32 prev) {
    const uint4 a0 = p4[0], a1 = p4[1], a2 = p4[2], a3 = p4[3];
    const u32 words[16] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w,
                           a2.x, a2.y, a2.z, a2.w, a3.x, a3.y, a3.z, a3.w};
    return line_start_mask_w(words, prev);
}

// The LDS window of parse_lines_k: every 64-byte segment is followed by one pad
// dword (17 dwords per segment), so the lanes of a wave, which read their own
// segments at about the same offset, hit 64 different banks instead of 4 (a
// 64-byte stride is 16 dwords). Bytes are read through a one-dword cache: one
// ds_read_b32 per 4 bytes of a line instead of one ds_read_u8 per byte. (With
// the window unpadded and read bytewise, the 16-way bank conflicts bounded the
// kernel at ~1.4 TB/s once the per-wave max-id atomic was gone.)
constexpr int PSW = PSEG / 4 + 1;                        // LDS dwords per segment
constexpr int PWIN = (int)(PCHUNK + PTAIL);              // window bytes
constexpr int PWIN_W = PWIN / PSEG * PSW;                // padded LDS dwords
struct LdsBytes {
    const u32* w;
    int64_t cq;
    u32 cw;
    __device__ __forceinline__ u32 operator[](int64_t p) {
        const int64_t q = p >> 2;
        if (q != cq) {
            cq = q;
            cw = w[q + (q >> 4)];
        }
        return (cw >> ((u32)(p & 3) * 8u)) & 0xFFu;
    }
};

// SWAR fast path of a line (8 bytes per register, no per-byte loop): the plain
// "digits blanks digits [blanks digits]" lines of an edge list, ids and weights of at
// most 9 digits (so no overflow check is needed: < 10^9 < ID_LIMIT). Anything else --
// signs, other blanks, a missing field, longer numbers -- falls back to the general
// `>> int` parser below, which also decides the error cases. After the last field
// the line is not looked at (extra columns are ignored, as by `>> int`).
constexpr u64 B_ONES = 0x0101010101010101ull;
constexpr u64 B_HIGH = 0x8080808080808080ull;
__device__ __forceinline__ u64 lds_load8(const u32* __restrict__ st, int p) {  // window bytes [p, p + 8)
    const int q = p >> 2, r = p & 3;
    const u32 d0 = st[q + (q >> 4)], d1 = st[q + 1 + ((q + 1) >> 4)], d2 = st[q + 2 + ((q + 2) >> 4)];
    const u32 lo = __builtin_amdgcn_alignbyte(d1, d0, (u32)r), hi = __builtin_amdgcn_alignbyte(d2, d1, (u32)r);
    return (u64)lo | ((u64)hi << 32);
}
__device__ __forceinline__ u64 nondigit_bits(u64 x) {  // bit 7 of every byte that is not '0'..'9'
    const u64 t = x ^ (0x30 * B_ONES);
    return ((((t & (0x7F * B_ONES)) + (0x76 * B_ONES)) | t) & B_HIGH);
}
__device__ __forceinline__ u64 nonzero_bits(u64 t) {  // bit 7 of every nonzero byte
    return ((((t & (0x7F * B_ONES)) + (0x7F * B_ONES)) | t) & B_HIGH);
}
__device__ __forceinline__ int lead_bytes(u64 flags) {  // bytes before the first flagged one
    return flags ? (int)(__builtin_ctzll(flags) >> 3) : 8;
}
__device__ __forceinline__ u32 digits8(u64 x, int nd) {  // value of the first nd (1..8) digits
    u64 d = (x & (0x0F * B_ONES)) << ((8 - nd) * 8);
    d = ((d * 2561ull) >> 8) & 0x00FF00FF00FF00FFull;
    d = ((d * 6553601ull) >> 16) & 0x0000FFFF0000FFFFull;
    return (u32)((d * 42949672960001ull) >> 32);
}
__device__ __forceinline__ bool fast_field(const u32* __restrict__ st, int& p, u32& val) {
    const u64 x = lds_load8(st, p);
    const int nd = lead_bytes(nondigit_bits(x));
    if (nd == 0) return false;
    if (nd < 8) {
        val = digits8(x, nd);
        p += nd;
        return true;
    }
    const u64 y = lds_load8(st, p + 8);
    const int n2 = lead_bytes(nondigit_bits(y));
    if (n2 > 1) return false;  // 10 digits or more
    val = digits8(x, 8);
    if (n2) val = val * 10u + (u32)(y & 0x0Fu);
    p += 8 + n2;
    return true;
}
__device__ __forceinline__ bool fast_sep(const u32* __restrict__ st, int& p) {  // 1..7 spaces / tabs
    const u64 x = lds_load8(st, p);
    const int nb = lead_bytes(nonzero_bits(x ^ (0x20 * B_ONES)) & nonzero_bits(x ^ (0x09 * B_ONES)));
    if (nb == 0 || nb == 8) return false;
    p += nb;
    return true;
}

// One `>> int` extraction from bytes t[0, len) (t: the LDS window of the
// block, or the whole text in global memory). 1 = read, 0 = failed on a
// non-blank (value 0), -1 = nothing but blanks before end of line, -2 = overflow.
template <typename T>
__device__ __forceinline__ int extract(T& t, int64_t len, int64_t& p, i64& out) {
    while (p < len && is_blank(t[p])) ++p;
    if (p >= len || t[p] == '\n') return -1;
    bool neg = false;
    u32 c = t[p];
    if (c == '+' || c == '-') {
        neg = (c == '-');
        ++p;
    }
    if (p >= len || !is_digit(t[p])) {
        out = 0;
        return 0;
    }
    // u32 accumulation: a value above 4294967295 is an overflow for every field
    // (ids are limited to ID_LIMIT, weights to the int range), so the digits
    // after it only need to be skipped
    u32 acc = 0;
    bool ovf = false;
    for (u32 d; p < len && is_digit(d = t[p]); ++p) {
        d -= '0';
        ovf |= acc > 429496729u || (acc == 429496729u && d > 5u);
        acc = acc * 10u + d;
    }
    if (ovf) return -2;
    out = neg ? -(i64)acc : (i64)acc;
    return 1;
}

// One line: `src dst [w]` with the reference's `>> int` semantics (:92-93).
// Returns false when the line is undefined behaviour for the reference.
template <typename T>
__device__ __forceinline__ bool parse_line(T& t, int64_t len, int64_t& p, bool weighted, i64& u, i64& v, i64& wt) {
    u = 0;
    v = 0;
    wt = 1;
    int r = extract(t, len, p, u);
    bool bad = (r != 1) || u > ID_LIMIT;
    if (!bad) {
        r = extract(t, len, p, v);
        bad = r < 0 || v < 0 || v > ID_LIMIT;
        if (!bad && weighted) {
            if (r == 0) wt = 0;  // stream failed: the weight extraction stores nothing -> 0
            else {
                const int r3 = extract(t, len, p, wt);
                bad = r3 < 0 || wt < 0;
            }
        }
    }
    return !bad;
}

__global__ __launch_bounds__(PB) void parse_count_k(const uint8_t* __restrict__ text, i64 len,
                                                    u32* __restrict__ block_cnt) {
    __shared__ u32 lds[PB / WAVE];
    const i64 seg = (i64)blockIdx.x * PCHUNK + (i64)threadIdx.x * PSEG;
    u32 c = 0;
    if (seg < len)
        c = (u32)__popcll(line_start_mask(reinterpret_cast<const uint4*>(text + seg),
                                          seg == 0 ? (u32)'\n' : (u32)text[seg - 1]));
    c = block_sum<PB / WAVE>(c, lds);
    if (threadIdx.x == 0) block_cnt[blockIdx.x] = c;
}

// The block's 16 KiB chunk plus a PTAIL-byte tail is loaded into LDS (padded
// layout, LdsBytes) with coalesced 16-byte loads; every lane then parses the lines
// that start in its 64-byte segment from LDS (byte loads from global were
// stride-64 across the wave: one cache line per lane per byte).
__global__ __launch_bounds__(PB) void parse_lines_k(const uint8_t* __restrict__ text, i64 len, int weighted,
                                                    const u64* __restrict__ block_off, u32* __restrict__ src,
                                                    u32* __restrict__ dst, u32* __restrict__ w,
                                                    u32* __restrict__ bmax, u64* __restrict__ errpos) {
    __shared__ u64 lds[PB / WAVE];
    __shared__ u32 lmax[PB / WAVE];
    __shared__ u32 stage[PWIN_W];
    const i64 base = (i64)blockIdx.x * PCHUNK;
    const uint4* g4 = reinterpret_cast<const uint4*>(text + base);
    for (int k = threadIdx.x; k < PWIN / 16; k += PB) {  // 16 window bytes -> 4 padded dwords
        const uint4 x = g4[k];
        u32* d = stage + 4 * k + (k >> 2);
        d[0] = x.x;
        d[1] = x.y;
        d[2] = x.z;
        d[3] = x.w;
    }
    __syncthreads();
    LdsBytes sb{stage, -1, 0u};
    // lines are parsed from the LDS window up to its end; a line that reaches the
    // end of the window is parsed again from global memory
    const int64_t wlen = min((i64)PWIN, len - base);
    const i64 seg = base + (i64)threadIdx.x * PSEG;
    u64 mask = 0;
    if (seg < len) {
        const u32 prev = seg == 0 ? (u32)'\n' : (threadIdx.x ? sb[(int64_t)threadIdx.x * PSEG - 1] : (u32)text[seg - 1]);
        const u32* sw = stage + threadIdx.x * PSW;
        u32 words[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) words[k] = sw[k];
        mask = line_start_mask_w(words, prev);
    }
    u64 tot;
    u64 idx = block_off[blockIdx.x] + block_excl_scan<PB / WAVE>((u64)__popcll(mask), lds, tot);
    i64 mx = -1;
    // (Staging a block's outputs through LDS for coalesced stores measured slower:
    // 1.32 against 1.20 ms on the K22 text.)
    while (mask) {
        const int b = __ffsll((long long)mask) - 1;
        mask &= mask - 1;
        const i64 start = seg + b;
        int64_t q = start - base;
        i64 u, v, wt;
        bool ok;
        int fp = (int)q;  // (a line start is < PCHUNK: the fast path's reads stay in the window)
        u32 fa, fb, fc = 1;
        if (fast_field(stage, fp, fa) && fast_sep(stage, fp) && fast_field(stage, fp, fb) &&
            (!weighted || (fast_sep(stage, fp) && fast_field(stage, fp, fc)))) {
            u = fa;
            v = fb;
            wt = fc;
            ok = true;
        } else {
            ok = parse_line(sb, wlen, q, weighted != 0, u, v, wt);
            if (q >= wlen && base + wlen < len) {  // ran into the window end: slow path
                int64_t pg = start;
                const uint8_t* tg = text;
                ok = parse_line(tg, len, pg, weighted != 0, u, v, wt);
            }
        }
        if (!ok) {
            atomicMin(errpos, (u64)start);
            u = 0;
            v = 0;
        }
        src[idx] = (u32)u;
        dst[idx] = (u32)v;
        if (w) w[idx] = (u32)wt;
        ++idx;
        mx = u > mx ? u : mx;
        mx = v > mx ? v : mx;
    }
    // the block's max id + 1 (0: no line) goes to its own slot: one word taking an
    // atomic from every wave saturates at ~88 per microsecond, which bounded this
    // kernel (K22 text: 524K waves, 6.1 ms)
    mx = wave_max(mx);
    if (lane_id() == 0) lmax[wave_id()] = (u32)(mx + 1);
    __syncthreads();
    if (threadIdx.x == 0) {
        u32 m = 0;
#pragma unroll
        for (int k = 0; k < PB / WAVE; ++k) m = max(m, lmax[k]);
        bmax[blockIdx.x] = m;
    }
}

// max over the per-block maxima (one block)
__global__ __launch_bounds__(1024) void max_blocks_k(const u32* __restrict__ bmax, i64 n, u64* __restrict__ out) {
    __shared__ u32 l[1024 / WAVE];
    u32 m = 0;
    for (i64 i = threadIdx.x; i < n; i += 1024) m = max(m, bmax[i]);
    m = wave_max(m);
    if (lane_id() == 0) l[wave_id()] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 0; k < 1024 / WAVE; ++k) m = max(m, l[k]);
        out[0] = m;
    }
}

}  // namespace

i64 padded_text_bytes(i64 len) { return (len + PCHUNK - 1) / PCHUNK * PCHUNK + PTAIL; }

ParseResult parse_snap_device(Ctx& ctx, const char* host_text, i64 len, bool weighted, DevBuf<u32>& src,
                              DevBuf<u32>& dst, DevBuf<u32>& w) {
    hipStream_t s = ctx.stream;
    const auto t0 = std::chrono::steady_clock::now();
    const i64 padded = padded_text_bytes(len);
    DevBuf<uint8_t> text((size_t)padded);
    PJ_HIP(hipMemsetAsync(text.p + len, 0, (size_t)(padded - len), s));
    if (len) PJ_HIP(hipMemcpyAsync(text.p, host_text, (size_t)len, hipMemcpyHostToDevice, s));
    PJ_HIP(hipStreamSynchronize(s));
    const double h2d_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ParseResult r = parse_device_text(ctx, text.p, len, weighted, src, dst, w);
    r.h2d_ms = h2d_ms;
    return r;
}

// text: len bytes on the device, zero-padded to padded_text_bytes(len)
ParseResult parse_device_text(Ctx& ctx, const uint8_t* text, i64 len, bool weighted, DevBuf<u32>& src,
                              DevBuf<u32>& dst, DevBuf<u32>& w) {
    hipStream_t s = ctx.stream;
    ParseResult r;
    const auto t1 = std::chrono::steady_clock::now();
    const i64 nblocks = (len + PCHUNK - 1) / PCHUNK;
    DevBuf<u32> bcnt((size_t)(nblocks > 0 ? nblocks : 1));  // line counts, then the blocks' max id + 1
    DevBuf<u64> boff((size_t)nblocks + 1);
    DevBuf<u64> scal(2);  // [0] = max id + 1, [1] = first bad byte offset
    ScanWs ws;
    if (nblocks) {
        parse_count_k<<<(unsigned)nblocks, PB, 0, s>>>(text, len, bcnt.p);
        PJ_LAUNCH_CHECK();
    }
    exclusive_scan_u32(bcnt.p, boff.p, nblocks, ws, s);
    u64 h[2] = {0ull, ~0ull};
    u64 total = 0;
    PJ_HIP(hipMemcpyAsync(&total, boff.p + nblocks, sizeof(u64), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipMemcpyAsync(scal.p, h, sizeof(h), hipMemcpyHostToDevice, s));
    PJ_HIP(hipStreamSynchronize(s));
    src.alloc((size_t)total);
    dst.alloc((size_t)total);
    if (weighted) w.alloc((size_t)total);
    if (nblocks && total) {
        parse_lines_k<<<(unsigned)nblocks, PB, 0, s>>>(text, len, weighted ? 1 : 0, boff.p, src.p, dst.p,
                                                      weighted ? w.p : nullptr, bcnt.p, scal.p + 1);
        PJ_LAUNCH_CHECK();
        max_blocks_k<<<1, 1024, 0, s>>>(bcnt.p, nblocks, scal.p);
        PJ_LAUNCH_CHECK();
    }
    PJ_HIP(hipMemcpyAsync(h, scal.p, sizeof(h), hipMemcpyDeviceToHost, s));
    PJ_HIP(hipStreamSynchronize(s));
    r.parse_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    r.nnz = (i64)total;
    r.max_id = (i64)h[0] - 1;
    if (h[1] != ~0ull) {  // error path: the line number from the text before the bad byte
        std::vector<char> pre((size_t)h[1]);
        if (h[1]) PJ_HIP(hipMemcpy(pre.data(), text, (size_t)h[1], hipMemcpyDeviceToHost));
        i64 line = 1;
        for (char c : pre) line += c == '\n';
        r.bad_line = line;
    }
    return r;
}

}  // namespace pj

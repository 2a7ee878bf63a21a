// jpegr_entropy.hip -- the reference's JPEG entropy stage on MI355X:
// per tile and channel, RLE of the zigzagged ints and a per-stream Huffman
// code built exactly as the reference builds it, then the encoded bits; and
// the inverse (decode + inverse RLE).  Algorithms/sequential/JPEG/JPEG.c:
//   RLE                        :767-808   (count, value) ints
//   calculate_frequency        :864-886   symbols in first-occurrence order
//   heapify / build_heap       :895-936   min-heap on count (strict <, left first)
//   build_huffman_tree         :938-962   pop, pop, APPEND the merged node and
//                                          heapify its leaf index (a no-op: the
//                                          node is not sifted up)
//   assign_codes               :964-983   DFS, left '0' / right '1'
//   generate_encoded_sequence  :993-1007
//   decode_huffman             :1009-1033; inverse_RLE :810-840
// The reference keeps codes as char strings and the sequence as '0'/'1'
// chars; here the bits are packed MSB-first and the code table is the list of
// (value, code length) in the reference's codes[] (DFS) order -- leaves of a
// full binary tree listed left to right, so the codes follow from the lengths
// (code[k] = (code[k-1] + 1) shifted to len[k]; left-aligned they increase).
//
// Mapping: one LANE per stream (a stream's Huffman build is a few hundred
// dependent steps; a wave per stream would issue each serial step for 64
// lanes).  A workgroup is one wave holding 64 tiles' streams of ONE channel,
// so Y (64 ints, ~100 RLE symbols) and chroma (32 ints) never share a wave.
// The per-lane working set lives in LDS laid out dword-column-per-lane (every
// lane owns its bank whatever index it uses).  The fast encoder
// (entropy_encode_lane) maps symbols through a direct per-lane table, so its
// RLE + count walk does one LDS round trip per position instead of a probe
// chain per symbol, and keeps each emission's leaf ids in registers for the
// sequence pass: 0.25 -> 0.14 ms per 4K image.  (A wave-cooperative RLE and
// sequence -- one stream per wave step, ballots and LDS atomics -- measured
// 0.34 ms: 64 dependent steps per wave, same-address atomics serialised.)
// Streams with a symbol outside the table or more than 24 (luma) / 12
// (chroma) distinct symbols (random 4K tiles: Y <= 21, chroma <= 10) are
// encoded by the chroma kernel after its own streams, with the hashed
// encoder (room for 128) over the wave's LDS.  Two kernels per call: luma,
// then chroma.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <type_traits>

#include "../../include/jpegr.h"

namespace {

constexpr int kLanes = 64;
constexpr int kFastCap = 24;             // distinct symbols in the LDS pass (luma)
constexpr int kChromaCap = 12;           // ... (chroma)
constexpr int kFullCap = 128;            // RLE of 64 ints: <= 128 symbols

// per-tile output layout
constexpr int kBitsPerTile = 256;        // bytes: [Y 128][Cr 64][Cb 64]
constexpr int kTablePerTile = 256;       // u32 entries: [Y 128][Cr 64][Cb 64]

__device__ __forceinline__ int stream_len(int c) { return c == 0 ? 64 : 32; }
__device__ __forceinline__ int coef_off(int c) { return c == 0 ? 0 : c == 1 ? 64 : 96; }
__device__ __forceinline__ int bits_off(int c) { return c == 0 ? 0 : c == 1 ? 128 : 192; }
__device__ __forceinline__ int bits_cap(int c) { return c == 0 ? 1024 : 512; }
// the reference's sequence buffers hold 1023 / 511 chars + NUL (JPEG.c:1248, :1286)
__device__ __forceinline__ int ref_bits_max(int c) { return c == 0 ? 1023 : 511; }

// Strided view of one lane's array: element i at p[i * stride].
template <typename T>
struct Col {
  T *p;
  int stride;
  __device__ __forceinline__ T &operator[](int i) const { return p[i * stride]; }
  __device__ __forceinline__ void clear(int n) const {
    for (int i = 0; i < n; ++i) p[i * stride] = 0;
  }
  // elements i, i + 1 (16-bit) as one word
  __device__ __forceinline__ uint32_t pair(int i) const {
    return (uint32_t)(uint16_t)p[i * stride] | ((uint32_t)(uint16_t)p[(i + 1) * stride] << 16);
  }
};

// One lane's array in LDS, dword-column layout: the lane owns dword column
// `lane` of a [rows][64] u32 block and packs 4 / sizeof(T) elements per
// dword, so every lane hits its own bank whatever index it uses (a plain
// [i][lane] byte column shares a dword between 4 lanes: up to 4-way
// conflicts under divergent indices).
template <typename T>
struct LCol {
  // Every access is type-punned over u32 storage (elements of 1, 2 or 4
  // bytes, pairs read as one dword): may_alias, or type-based alias analysis
  // lets the compiler move a dword read above a half-word store of the same
  // word (it did, once a sift was unrolled without branches).
  typedef T __attribute__((may_alias)) TA;
  typedef uint32_t __attribute__((may_alias)) WA;
  uint8_t *p;                                   // &block[0][lane] as bytes
  // (indices are never negative: unsigned division is a shift and a mask)
  __device__ __forceinline__ TA &operator[](int i) const {
    constexpr uint32_t per = 4 / sizeof(T);
    const uint32_t u = (uint32_t)i;
    return *reinterpret_cast<TA *>(p + (u / per) * (4 * kLanes) + (u % per) * sizeof(T));
  }
  // zero elements [0, n) (n a multiple of 4 / sizeof(T)): whole dwords
  __device__ __forceinline__ void clear(int n) const {
    constexpr int per = 4 / (int)sizeof(T);
    for (int i = 0; i < n / per; ++i) *reinterpret_cast<WA *>(p + i * (4 * kLanes)) = 0u;
  }
  // 16-bit elements i, i + 1 (i even: one dword, one LDS read)
  __device__ __forceinline__ uint32_t pair(int i) const {
    return *reinterpret_cast<const WA *>(p + (i / 2) * (4 * kLanes));
  }
};

// One lane's working set for a stream with at most Cap distinct symbols.
template <template <typename> class A>
struct Work {
  static constexpr bool kPackLen = false;
  static constexpr bool kTopDown = false;
  A<int16_t> sym;       // [Cap]       leaf -> symbol value (the int, without +1000)
  A<uint8_t> hash;      // [Hash]      open-addressing map symbol -> leaf + 1 (0 = empty)
  A<uint16_t> heap;     // [Cap + 2]   heap entry i (count << 8 | node id) at slot i + 1,
                        //             so that children 2i+1, 2i+2 share a dword; merged
                        //             node m's children (left | right << 8) at entry
                        //             U - 1 - m, the slot the heap frees as it shrinks
  A<uint32_t> code;     // [Cap]       leaf code bits (right-aligned)
  A<uint8_t> len;       // [Cap]       leaf code length
  A<uint16_t> stk;      // [Cap + 1]   DFS stack: node | depth << 8
};

// Sift x down from index i (JPEG.c:895-911: smallest of i, left, right by
// count with strict <, left tested first), moving children up into the hole
// -- the same final arrangement as the reference's swaps.  x is passed in
// registers (slot i is not read), and each LDS round trip serves two levels:
// the children pair and both grandchildren pairs are read together.  Slots
// past MaxSlot (the array's last even slot) are clamped: such a pair is never
// used.  Returns the entry left at index i (for the root: the new minimum).
template <int MaxSlot, class W>
__device__ __forceinline__ uint16_t sift(const W &w, int size, int i, uint16_t x) {
  const int cx = x >> 8;
  uint16_t top = x;
  bool moved = false;
  for (;;) {
    const int l = 2 * i + 1, r = l + 1;
    if (l >= size) break;
    const uint32_t pc = w.heap.pair(l + 1);               // entries l, r (slots l + 1, l + 2)
    const uint32_t pgl = w.heap.pair(min(2 * l + 2, MaxSlot));   // l's children
    const uint32_t pgr = w.heap.pair(min(2 * l + 4, MaxSlot));   // r's children
    const uint16_t hl = (uint16_t)pc, hr = (uint16_t)(pc >> 16);
    int s = i, cs = cx;
    uint16_t hs = x;
    if ((hl >> 8) < cs) { s = l; cs = hl >> 8; hs = hl; }
    if (r < size && (hr >> 8) < cs) { s = r; hs = hr; }
    if (s == i) break;
    w.heap[i + 1] = hs;
    if (!moved) top = hs;
    moved = true;
    i = s;
    const int l2 = 2 * i + 1;                             // the next level, prefetched
    if (l2 >= size) break;
    const uint32_t pg = s == l ? pgl : pgr;
    const uint16_t gl = (uint16_t)pg, gr = (uint16_t)(pg >> 16);
    int s2 = i, c2 = cx;
    uint16_t h2 = x;
    if ((gl >> 8) < c2) { s2 = l2; c2 = gl >> 8; h2 = gl; }
    if (l2 + 1 < size && (gr >> 8) < c2) { s2 = l2 + 1; h2 = gr; }
    if (s2 == i) break;
    w.heap[i + 1] = h2;
    i = s2;
  }
  w.heap[i + 1] = x;
  return top;
}

// The same sift for heaps of at most Cap <= 32 entries, branch-free: a fixed
// floor(log2(Cap)) levels (the deepest any sift can go), two per LDS round
// trip, a done flag instead of a break.  Once x has landed, the remaining
// levels rewrite x at its index (idempotent).  The loop form above paid the
// exec-mask bookkeeping of every lane's own exit at every level.
template <int Cap, int kDepth, class W>
__device__ __forceinline__ uint16_t sift_depth(const W &w, int size, int i, uint16_t x,
                                               int *fi = nullptr) {
  constexpr int kMaxSlot = Cap & ~1;
  static_assert(Cap <= 31 && kDepth >= 1 && kDepth <= 4, "fixed depth");
  // counts compare as whole entries against a count with a zero id byte
  // (strict <): e < (c << 8) iff e >> 8 < c
  const uint32_t xk = x & 0xFF00u;
  uint16_t top = x;
  bool done = false;
#pragma unroll
  for (int d = 0; d < kDepth; d += 2) {
    const int l = 2 * i + 1, r = l + 1;
    const uint32_t pc = w.heap.pair(min(l + 1, kMaxSlot));      // entries l, r
    const uint32_t pgl = w.heap.pair(min(2 * l + 2, kMaxSlot));  // l's children
    const uint32_t pgr = w.heap.pair(min(2 * l + 4, kMaxSlot));  // r's children
    {
      const uint32_t hl = pc & 0xFFFFu, hr = pc >> 16;
      const bool tl = l < size && hl < xk;
      const uint32_t ck = tl ? (hl & 0xFF00u) : xk;
      const bool tr = r < size && hr < ck;
      const bool mv = !done && (tl || tr);
      const uint16_t hs = (uint16_t)(tr ? hr : hl);
      if (d == 0) top = mv ? hs : x;
      w.heap[i + 1] = mv ? hs : x;
      done = !mv;
      i = mv ? (tr ? r : l) : i;
    }
    if (d + 1 < kDepth) {
      const uint32_t pg = i == r ? pgr : pgl;                 // (unused once done)
      const int l2 = 2 * i + 1, r2 = l2 + 1;
      const uint32_t gl = pg & 0xFFFFu, gr = pg >> 16;
      const bool tl = l2 < size && gl < xk;
      const uint32_t ck = tl ? (gl & 0xFF00u) : xk;
      const bool tr = r2 < size && gr < ck;
      const bool mv = !done && (tl || tr);
      w.heap[i + 1] = mv ? (uint16_t)(tr ? gr : gl) : x;
      done = !mv;
      i = mv ? (tr ? r2 : l2) : i;
    }
  }
  w.heap[i + 1] = x;
  if (fi) *fi = i;                                    // where x landed
  return top;
}

template <int Cap, class W>
__device__ __forceinline__ uint16_t sift_fixed(const W &w, int size, int i, uint16_t x) {
  constexpr int kDepth = Cap >= 16 ? 4 : Cap >= 8 ? 3 : Cap >= 4 ? 2 : 1;   // floor(log2 Cap)
  return sift_depth<Cap, kDepth>(w, size, i, x);
}

// The same with the depth cut to what a wave-uniform bound allows: no lane
// of the wave sifts more than `levels` levels (a uniform branch picks the
// unrolled depth).
// levels a sift from index i can descend in a heap of at most s entries
__host__ __device__ constexpr int sift_levels_bound(int s, int i) {
  int d = 0;
  for (int j = i; 2 * j + 1 < s; j = 2 * j + 1) ++d;
  return d;
}

// build_heap's sifts (JPEG.c:913-936) from index I down to 0, unrolled so
// that each sift's x is the entry's initial value from registers: a sift
// from a later index moves only entries of that index's subtree, which holds
// no earlier index.  Returns, through root, the entry left at index 0.
template <int Cap, int I, class W>
__device__ __forceinline__ void build_heap_from(const W &w, int umax, int U,
                                                const uint32_t *h0, uint16_t &root) {
  if constexpr (I >= 0) {
    if (I < umax / 2) {                                 // uniform
      if (I < U / 2) {
        // the depth of index I in a heap of Cap: the levels of the wave's
        // own heaps (umax) are the same for all but small streams
        const uint16_t t =
            sift_depth<Cap, sift_levels_bound(Cap, I)>(w, U, I, (uint16_t)h0[I]);
        if (I == 0) root = t;
      }
    }
    build_heap_from<Cap, I - 1>(w, umax, U, h0, root);
  }
}

template <int Cap, class W>
__device__ __forceinline__ uint16_t sift_any(const W &w, int size, int i, uint16_t x) {
  if constexpr (Cap <= 31) return sift_fixed<Cap>(w, size, i, x);
  else return sift<Cap & ~1>(w, size, i, x);
}

// The Huffman code of one stream from its U symbols' counts, exactly as the
// reference builds it: build_heap (JPEG.c:913-936) over the frequency list in
// first-occurrence order, build_huffman_tree (:938-962: pop, pop, append the
// merged node WITHOUT sifting it up), assign_codes (:964-983: DFS, left
// first).  In: w.heap[u + 1] = count << 8 | u and w.sym[u] for u < U.  Out:
// w.code / w.len per leaf and the table (value | length << 16 per code, DFS
// order).  Returns true when a code exceeds the reference's char code[32].
// h0 (Cap <= 31): heap entry i's initial value (count << 8 | i) for i < U.
template <int Cap, class W>
__device__ __forceinline__ bool tree_codes(const W &w, int U, uint32_t *__restrict__ table,
                                           const uint32_t *h0 = nullptr) {
  int size = U, next = U;
  uint16_t root;
  int umax = 0;
  if constexpr (Cap <= 31) {
    // Every lane's heap shrinks by one per merge, so at merge step t no lane's
    // heap exceeds Umax - t (Umax: the wave's largest U): each sift runs only
    // the levels that bound allows (and build_heap's sift from index i, the
    // levels below i in a heap of Umax), picked by uniform branches.
#pragma unroll
    for (int b = 4; b >= 0; --b)
      if (__ballot(U >= (umax | (1 << b)))) umax |= 1 << b;
    root = (uint16_t)h0[0];
    build_heap_from<Cap, Cap / 2 - 1>(w, umax, U, h0, root);
    // Each pop moves the last entry to the root and sifts it.  The first pop's
    // last entry is the node the previous merge appended (in registers); the
    // second pop's is read before the first sift, which changes that index
    // (the heap's last: no children) only by landing its x there.  So each
    // merge waits on the two sifts' LDS round trips alone.
    uint16_t last = w.heap[U];                        // entry U - 1 after the build
    // Merge step t pops from heaps of at most umax - t - 1 entries: the steps
    // run in phases of one sift depth, floor(log2(umax - t - 1)) levels (the
    // second pop's heap is one smaller: the same depth serves), so no step
    // dispatches on its depth or loops to find it.
    auto merge = [&](auto depth) {
      constexpr int D = decltype(depth)::value;
      if (size > 1) {
        const uint16_t left = root;
        --size;
        const uint16_t e2 = w.heap[size];             // entry size - 1, before the sift
        int fi;
        root = sift_depth<Cap, D>(w, size, 0, last, &fi);
        const uint16_t right = root;
        const uint16_t x2 = fi == size - 1 ? last : e2;
        --size;
        root = sift_depth<Cap, D>(w, size, 0, x2);
        const uint16_t merged = (uint16_t)((((left >> 8) + (right >> 8)) << 8) | next);
        w.heap[size + 1] = merged;                                              // not sifted up
        last = merged;
        if constexpr (W::kTopDown) {
          // record of merged node m = next - U: left | right << 6 | leaves
          // under it << 12 | leaves under left << 17 (| DFS position << 22 |
          // depth << 27, or-ed in top-down)
          const int li = left & 255, ri = right & 255;
          const uint32_t rl = w.mrec[li < U ? 0 : li - U], rr = w.mrec[ri < U ? 0 : ri - U];
          const uint32_t nl = li < U ? 1u : (rl >> 12) & 31u, nr = ri < U ? 1u : (rr >> 12) & 31u;
          w.mrec[next - U] = (uint32_t)li | (uint32_t)ri << 6 | (nl + nr) << 12 | nl << 17;
        } else {
          w.heap[U - (next - U)] = (uint16_t)((left & 255) | ((right & 255) << 8));   // freed slot
        }
        ++size;
        ++next;
        if (size == 1) root = merged;
      }
    };
    int t = 0;
    if constexpr (Cap >= 17) {
      for (; umax - t - 1 >= 16; ++t) merge(std::integral_constant<int, 4>{});
    }
    if constexpr (Cap >= 9) {
      for (; umax - t - 1 >= 8; ++t) merge(std::integral_constant<int, 3>{});
    }
    for (; umax - t - 1 >= 4; ++t) merge(std::integral_constant<int, 2>{});
    for (; umax - t > 1; ++t) merge(std::integral_constant<int, 1>{});
  } else {
  for (int i = U / 2 - 1; i >= 0; --i) sift_any<Cap>(w, U, i, w.heap[i + 1]);
  root = w.heap[1];
  while (size > 1) {
    // pop, pop (the moved last entry sifted from the root; the new root is
    // known in registers), append the merged node unsifted
    const uint16_t left = root;
    --size;
    root = sift_any<Cap>(w, size, 0, w.heap[size + 1]);
    const uint16_t right = root;
    --size;
    root = sift_any<Cap>(w, size, 0, w.heap[size + 1]);
    const uint16_t merged = (uint16_t)((((left >> 8) + (right >> 8)) << 8) | next);
    w.heap[size + 1] = merged;                                              // not sifted up
    w.heap[U - (next - U)] = (uint16_t)((left & 255) | ((right & 255) << 8));   // freed slot
    ++size;
    ++next;
    if (size == 1) root = merged;
  }
  }

  // ---- codes: DFS, left first (JPEG.c:964-983) ------------------------------
  // Leaves pop in codes[] order; each code follows from the previous one:
  // code[k] = (code[k-1] + 1) moved to length len[k].  The current node stays
  // in registers: an internal node stacks its right child and descends left.
  bool over = false;
  if constexpr (W::kTopDown) {
    // Top-down instead of the DFS: merged nodes from the root down (merge
    // step t's node is m = U - 2 - t), each handing its children their depth
    // and DFS position (left: the parent's; right: + the leaves under left);
    // a leaf records (depth | leaf << 8) at its position.  U - 1 steps
    // instead of 2U - 1.  Then the leaves in DFS order give the codes as the
    // DFS does.
    static_assert(2 * Cap - 1 <= 64 && Cap <= 31, "record fields");
    if (U == 1) w.dep[0] = 0;                         // the root is leaf 0, depth 0
    for (int t = 0; t + 1 < umax; ++t) {
      if (t + 1 < U) {
        const uint32_t rc = w.mrec[U - 2 - t];
        const int li = (int)(rc & 63u), ri = (int)((rc >> 6) & 63u);
        const uint32_t pos = (rc >> 22) & 31u, dc = (rc >> 27) + 1u, nl = (rc >> 17) & 31u;
        if (li < U) w.dep[(int)pos] = (uint16_t)(dc | (uint32_t)li << 8);
        else atomicOr(&w.mrec[li - U], pos << 22 | dc << 27);
        if (ri < U) w.dep[(int)(pos + nl)] = (uint16_t)(dc | (uint32_t)ri << 8);
        else atomicOr(&w.mrec[ri - U], (pos + nl) << 22 | dc << 27);
      }
    }
    int plen = 0;
    uint32_t pcode = 0;
    uint32_t de[Cap];
    int sy[Cap];
    // (all Cap positions, no uniform branch per position: past a lane's U
    // the entries are dead rows' values and nothing is stored)
#pragma unroll
    for (int k = 0; k < Cap; ++k) de[k] = w.dep[k];
#pragma unroll
    for (int k = 0; k < Cap; ++k) sy[k] = w.sym[min((int)(de[k] >> 8), Cap - 1)];
#pragma unroll
    for (int k = 0; k < Cap; ++k) {
      const int d = (int)(de[k] & 255u), x = min((int)(de[k] >> 8), Cap - 1);
      const uint32_t t = k ? pcode + 1 : 0u;
      pcode = d >= plen ? t << (d - plen) : t >> (plen - d);
      plen = d;
      if (k < U) {
        // the code left-aligned, its length in the low 5 bits (depth <= Cap - 1
        // < 27 leaves them zero)
        w.code[x] = (d ? pcode << (32 - d) : 0u) | (uint32_t)d;
        table[k] = (uint16_t)sy[k] | ((uint32_t)d << 16);
      }
    }
    return over;
  } else {
  int sp = 0, k = 0, plen = 0;
  uint32_t pcode = 0;
  int e = root & 255;                                 // the root, depth 0
  // Both successors (the stack top, the node's children) and a leaf's symbol
  // are read at the top of every step, one LDS round trip, so a leaf step
  // does not wait on a second one before its table store.
  for (;;) {
    const int x = e & 255, d = e >> 8;
    const bool leaf = x < U;
    const int top = w.stk[sp > 0 ? sp - 1 : 0];       // a leaf's successor
    const int ch = w.heap[leaf ? 0 : 2 * U - x];      // children of merged node x - U
    const int sy = w.sym[leaf ? x : 0];               // a leaf's symbol
    if (leaf) {                                       // leaf: next entry of codes[]
      const uint32_t t = k ? pcode + 1 : 0u;
      pcode = d >= plen ? t << (d - plen) : t >> (plen - d);
      plen = d;
      if constexpr (W::kPackLen) {
        w.code[x] = pcode | (uint32_t)d << 24;        // depth <= Cap - 1 < 24
      } else {
        w.code[x] = pcode;
        w.len[x] = (uint8_t)d;
      }
      if (d > 31) over = true;                        // char code[32] (JPEG.c:861)
      table[k] = (uint16_t)sy | ((uint32_t)d << 16);
    } else {
      w.stk[sp] = (uint16_t)((ch >> 8) | ((d + 1) << 8));     // right, visited later
    }
    if (leaf && sp == 0) break;
    k += leaf ? 1 : 0;
    sp += leaf ? -1 : 1;
    e = leaf ? top : (ch & 255) | ((d + 1) << 8);              // left now
  }
  return over;
  }
}

enum : int { kOk = 0, kDefer = 1, kOverflow = 2 };

__device__ __forceinline__ int hash_slot(int s, int mask) {
  return (int)(((uint32_t)(s + 1024) * 0x9E3779B1u) >> 24) & mask;
}

// The RLE of the n ints at zz (JPEG.c:767-808): emit(count), emit(value) at
// the end of every run, in order.  The ints are read 8 at a time as 16-B
// loads, the next chunk in flight while this one is walked (a lane's stream
// is 128 or 64 contiguous bytes: one load per int, 64 lanes 256 B apart,
// was a memory round trip per int).
template <class F>
__device__ __forceinline__ void rle_walk(const int16_t *__restrict__ zz, int n, F &&emit) {
  const uint4 *src = reinterpret_cast<const uint4 *>(zz);
  uint4 nxt = src[0];
  int cur = 0, run = 0;
  for (int ch = 0; ch < n / 8; ++ch) {
    const uint4 q = nxt;
    if (ch + 1 < n / 8) nxt = src[ch + 1];
    const uint32_t wv[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int v = (int16_t)(wv[j >> 1] >> (16 * (j & 1)));
      if (ch == 0 && j == 0) {
        cur = v;
        run = 1;
      } else if (v == cur) {
        ++run;
      } else {
        emit(run);
        emit(cur);
        cur = v;
        run = 1;
      }
    }
  }
  emit(run);
  emit(cur);
}

// Encode one stream of n ints at zz (global).  Writes the packed bits (slot
// of cap_bits), the table (value | len << 16 per code, DFS order) and the
// meta word (nbits | rle_len << 16 | ncodes << 24).  Returns kOk, kDefer
// (more than Cap distinct symbols; nothing written) or kOverflow (a code or
// the sequence exceeds the reference's fixed buffers; written truncated).
template <int Cap, int Hash, class W>
__device__ int encode_stream(const int16_t *__restrict__ zz, int n, const W &w,
                             uint8_t *__restrict__ bits, int cap_bits, int ref_max,
                             uint32_t *__restrict__ table, uint32_t *__restrict__ meta) {
  static_assert((Hash & (Hash - 1)) == 0 && Hash >= Cap * 4 / 3, "power of two, load <= 3/4");
  constexpr int kMask = Hash - 1;
  // symbol -> leaf through the hash (inserting new symbols in first-occurrence
  // order, JPEG.c:864-886); returns -1 when a new symbol does not fit
  int U = 0;
  auto leaf_of = [&](int s, bool insert) -> int {
    int h = hash_slot(s, kMask);
    for (;;) {
      const int e = w.hash[h];
      if (e == 0) {
        if (!insert || U == Cap) return -1;
        w.hash[h] = (uint8_t)(U + 1);
        w.sym[U] = (int16_t)s;
        w.heap[U + 1] = (uint16_t)U;                // count 0, id U
        return U++;
      }
      if (w.sym[e - 1] == s) return e - 1;
      h = (h + 1) & kMask;
    }
  };
  w.hash.clear(Hash);

  // ---- RLE (JPEG.c:767-808) + frequencies --------------------------------------
  int R = 0;
  bool defer = false;
  auto count = [&](int s) {
    const int u = leaf_of(s, true);
    if (u < 0) {
      defer = true;
      return;
    }
    w.heap[u + 1] = (uint16_t)(w.heap[u + 1] + 256);
    ++R;
  };
  rle_walk(zz, n, [&](int sy) {
    if (!defer) count(sy);
  });
  if (defer) return kDefer;

  // ---- heap, tree and codes (JPEG.c:913-983) ---------------------------------
  bool over = tree_codes<Cap>(w, U, table);

  // ---- encoded sequence, MSB-first (JPEG.c:993-1007): RLE again --------------
  uint64_t acc = 0;
  int nacc = 0, nbits = 0, word = 0;
  const int nwords = cap_bits / 32;
  uint32_t *wout = reinterpret_cast<uint32_t *>(bits);
  auto put = [&](int s) {
    const int leaf = leaf_of(s, false);
    const int L = w.len[leaf];
    if (L > 32) return;                               // flagged above; no 64-bit overshift
    acc = (acc << L) | w.code[leaf];
    nacc += L;
    nbits += L;
    if (nacc >= 32) {
      const uint32_t v = (uint32_t)(acc >> (nacc - 32));
      if (word < nwords) wout[word] = __builtin_bswap32(v);
      ++word;
      nacc -= 32;
    }
  };
  rle_walk(zz, n, put);
  if (nacc && word < nwords) wout[word] = __builtin_bswap32((uint32_t)(acc << (32 - nacc)));
  if (nbits > ref_max) over = true;                   // char sequence[1024] / [512]
  *meta = (uint32_t)(nbits < 0xFFFF ? nbits : 0xFFFF) | ((uint32_t)R << 16) |
          ((uint32_t)U << 24);
  return over ? kOverflow : kOk;
}

template <typename T>
using GColT = Col<T>;

// Scratch (d_scratch): per luma wave a list of its deferred streams (64
// entries), then per luma wave a word deferred | overflowed << 8 (lanes).
// The chroma kernel reads them (its even wave 2 v: luma wave v), so no
// kernel runs before the lane kernels or after them.

// ---- the fast encoder: one lane per stream, no probing ------------------------
// Symbols index a direct per-lane table (symbol + kOff -> leaf + 1, u8), so a
// lookup is one LDS read with no probe loop: the RLE walk is unrolled over
// the stream's positions and, per position, every lane whose run ends there
// looks up BOTH its symbols (count, value) with the two reads in flight
// together (an equal pair is resolved in registers) -- one LDS round trip
// per position, where the hashed walk took up to three per symbol, for the
// wave's longest probe chain.  Counts are bumped by ds_add_u32 on the heap
// entry's half-word (no read).  Each emission's two leaf ids stay in
// registers (5 bits each, 3 positions per dword), so the sequence pass reads
// only the codes.  The table is dead after the count: the DFS stack and the
// codes overlay it.  A stream with a symbol outside the table or more than
// Cap distinct symbols is deferred: the chroma kernel encodes it with the
// hashed encoder after its own streams.
template <int N>
struct LaneLds {
  static constexpr int Cap = N == 64 ? kFastCap : kChromaCap;
  static constexpr int Keys = N == 64 ? 176 : 120;   // symbols [-Off, Keys - Off)
  static constexpr int Off = N == 64 ? 64 : 48;       // counts: 1 .. N
  static constexpr int StkRows = (Cap + 2) / 2;       // overlays of the table (dword rows)
  // a zero row, then per leaf its code left-aligned | length (leaf + 1
  // indexes from the zero row: id 0, no emission, reads a length-0 code);
  // past the codes, the sequence pass's bit rows (through heap and sym)
  static constexpr int ZeroRow = StkRows, CodeRow = StkRows + 1;
  static_assert(CodeRow + Cap <= Keys / 4, "stack and codes fit the table");
  // (the merge records, Cap - 1 rows from row 0, are dead before the codes
  // and the zero row are written; the depths by DFS position take Cap / 2
  // rows of the dead heap)
  static_assert(Off + N < Keys, "every count is a key");
  // Luma's heap takes a dword row per entry (no half-word address arithmetic
  // in the sifts; 19 KB per wave, still 8 waves per CU: a 4K image's 2,025
  // luma waves in one round); chroma's stays two entries per dword (10 KB:
  // 16 waves per CU, its 4,050 waves in one round).
  static constexpr bool Wide = N == 64;
  static constexpr int HeapRows = Wide ? Cap + 2 : (Cap + 2) / 2;
  static_assert(HeapRows >= Cap / 2, "the walk's (symbol | count) rows");
  uint32_t tab[Keys / 4][kLanes];
  uint32_t heap[HeapRows][kLanes];
  uint32_t sym[Cap / 4][kLanes];                      // int8 symbols
};

// One lane's u16 array with an element per dword row (the low half); a pair
// is two rows
struct WCol {
  typedef uint16_t __attribute__((may_alias)) TA;
  typedef uint32_t __attribute__((may_alias)) WA;
  uint8_t *p;
  __device__ __forceinline__ TA &operator[](int i) const {
    return *reinterpret_cast<TA *>(p + (uint32_t)i * (4 * kLanes));
  }
  __device__ __forceinline__ uint32_t pair(int i) const {
    const WA *q = reinterpret_cast<const WA *>(p + (uint32_t)i * (4 * kLanes));
    return __builtin_amdgcn_perm(q[kLanes], q[0], 0x05040100u);
  }
};

template <class HeapCol>
struct LaneWork {                                     // the arrays tree_codes uses
  static constexpr bool kPackLen = true;              // code and length in one dword (tree_codes)
  static constexpr bool kTopDown = true;              // codes top-down over mrec (tree_codes)
  LCol<int8_t> sym;
  HeapCol heap;
  LCol<uint32_t> code;
  LCol<uint32_t> mrec;   // merged node m's record (the dead table's rows, before the codes)
  LCol<uint16_t> dep;    // (depth | leaf << 8) by DFS position (the dead heap's rows)
};

template <bool kLuma>
__global__ __launch_bounds__(kLanes) void entropy_encode_lane(
    const int16_t *__restrict__ coef, size_t ntiles, uint8_t *__restrict__ bits,
    uint32_t *__restrict__ meta, uint32_t *__restrict__ table, uint32_t *__restrict__ lists,
    uint32_t *__restrict__ status) {
  constexpr int N = kLuma ? 64 : 32;
  using L = LaneLds<N>;
  constexpr int Cap = L::Cap, Keys = L::Keys, Off = L::Off;
  __shared__ L S;
  const int lane = threadIdx.x;
  const int c = kLuma ? 0 : 1 + (int)(blockIdx.x & 1);      // channel of this wave
  const size_t tile = (size_t)(kLuma ? blockIdx.x : blockIdx.x >> 1) * kLanes + lane;
  // (luma wave 0: the overflow count starts here; every later count is
  // added by the chroma kernel)
  if (kLuma && blockIdx.x == 0 && lane == 0) status[0] = 0;
  if (tile >= ntiles) return;
  // luma wave v's list and word (see the scratch layout above)
  const size_t lv = kLuma ? blockIdx.x : blockIdx.x >> 1;
  const size_t nlw = (ntiles + kLanes - 1) / kLanes;
  uint32_t *const lst = lists + lv * kLanes;
  uint32_t *const lword = lists + nlw * kLanes + lv;
  auto colp = [&](uint32_t *row0) { return reinterpret_cast<uint8_t *>(row0 + lane); };
  uint8_t *const tabc = colp(&S.tab[0][0]);
  using HeapCol = typename std::conditional<L::Wide, WCol, LCol<uint16_t>>::type;
  const LaneWork<HeapCol> w{{colp(&S.sym[0][0])}, {colp(&S.heap[0][0])},
                            {colp(&S.tab[L::CodeRow][0])}, {colp(&S.tab[0][0])},
                            {colp(&S.heap[0][0])}};

  // the stream: N int16 as N / 2 packed dwords (16-B loads)
  uint32_t iw[N / 2];
  {
    const uint4 *src = reinterpret_cast<const uint4 *>(coef + tile * 128 + coef_off(c));
#pragma unroll
    for (int k = 0; k < N / 8; ++k) {
      const uint4 q = src[k];
      iw[4 * k] = q.x; iw[4 * k + 1] = q.y; iw[4 * k + 2] = q.z; iw[4 * k + 3] = q.w;
    }
  }
#pragma unroll
  for (int r = 0; r < Keys / 4; ++r) *reinterpret_cast<uint32_t *>(tabc + r * (4 * kLanes)) = 0u;
  auto val = [&](int i) { return (int)(int16_t)(iw[i >> 1] >> (16 * (i & 1))); };
  auto tab_at = [&](int k) -> uint8_t & {
    return *(tabc + (k >> 2) * (4 * kLanes) + (k & 3));
  };
  auto row = [&](int r) {                            // dword row r of the heap rows
    return reinterpret_cast<uint32_t *>(w.heap.p + r * (4 * kLanes));
  };

  // ---- RLE (JPEG.c:767-808) + frequencies (JPEG.c:864-886) ------------------
  // run k ends at position i when i == N - 1 or the next int differs; it
  // emits (count, value).  Leaf ids in first-occurrence order.
  uint32_t lid[(N + 2) / 3];             // per position: (leaf_c + 1) | (leaf_v + 1) << 5
#pragma unroll
  for (int j = 0; j < (N + 2) / 3; ++j) lid[j] = 0;
  int U = 0, start = 0, R = 0;
  bool defer = false;
  // One exec region per position and no branch inside it: the stores are
  // unconditional and idempotent (a known symbol rewrites its table entry and
  // its symbol with the values they hold), and a count is a ds_add into the
  // zeroed heap rows, which hold (symbol | count << 8) per leaf during the
  // walk.  A stream that must be deferred runs on with clamped leaf ids over
  // its own columns (the results are dropped).
#pragma unroll
  for (int r = 0; r < Cap / 2; ++r) *row(r) = 0u;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int v = val(i);
    const bool end = i == N - 1 || val(i + 1 < N ? i + 1 : i) != v;
    if (end) {
      const int kc = i + 1 - start + Off;
      start = i + 1;
      const bool bad = (uint32_t)(v + Off) >= (uint32_t)Keys;
      const int kv = bad ? kc : v + Off;
      const int ec = tab_at(kc), ev = tab_at(kv);       // both reads in flight
      const bool same = kv == kc;
      const int lc = ec ? ec - 1 : U;
      const int nu = U + (ec ? 0 : 1);
      const int lv = same ? lc : (ev ? ev - 1 : nu);
      const int nu2 = nu + ((same || ev) ? 0 : 1);
      defer = defer || bad || nu2 > Cap;
      const int lcw = min(lc, Cap - 1), lvw = min(lv, Cap - 1);
      tab_at(kc) = (uint8_t)(lcw + 1);
      tab_at(kv) = (uint8_t)(lvw + 1);
      // leaf u's symbol and count: one u16 (symbol | count << 8) at half
      // u & 1 of dword row u >> 1, so the store and the add share an address
      uint8_t *const sc = w.heap.p + ((lcw >> 1) << 8), *const sv = w.heap.p + ((lvw >> 1) << 8);
      const int hc = (lcw & 1) << 4, hv = (lvw & 1) << 4;
      const bool fc = ec == 0, fv = !same && ev == 0;    // first occurrences
      const uint32_t ac = (fc ? (uint32_t)(uint8_t)(kc - Off) : 0u) + ((same ? 2u : 1u) << 8);
      const uint32_t av = (fv ? (uint32_t)(uint8_t)(kv - Off) : 0u) + ((same ? 0u : 1u) << 8);
      atomicAdd(reinterpret_cast<uint32_t *>(sc), ac << hc);
      atomicAdd(reinterpret_cast<uint32_t *>(sv), av << hv);
      U = min(nu2, Cap);
      R += 2;                                         // the run's (count, value)
      lid[i / 3] |= (uint32_t)((lcw + 1) | ((lvw + 1) << 5)) << (10 * (i % 3));
    }
  }
  uint64_t dm = 0;                                    // (luma) the wave's deferred lanes
  if constexpr (kLuma) {
    const uint64_t act = __ballot(1);
    dm = __ballot(defer);
    if (defer) lst[__popcll(dm & ((1ull << lane) - 1ull))] = (uint32_t)(tile * 3 + c);
    if (dm == act) {                                  // (no lane left to report at the end)
      if (lane == __builtin_ctzll(act)) *lword = (uint32_t)__popcll(dm);
      return;
    }
    if (defer) return;
  } else {
    dm = __ballot(defer);                             // encoded below, after the fast path
  }
  if (!defer) {                                       // (luma: every lane left)
    // (symbol | count << 8) per leaf -> the symbols (i8, 4 per dword) and the
    // heap entries (count << 8 | leaf at slot leaf + 1)
    uint32_t h0[Cap];                                   // heap entry u: count << 8 | u
    {
      uint32_t sc[Cap / 2];
#pragma unroll
      for (int k = 0; k < Cap / 2; ++k) sc[k] = *row(k);
#pragma unroll
      for (int u = 0; u < Cap; ++u) h0[u] = ((sc[u >> 1] >> (16 * (u & 1))) & 0xFF00u) | (uint32_t)u;
#pragma unroll
      for (int j = 0; j < Cap / 4; ++j)
        *reinterpret_cast<uint32_t *>(w.sym.p + j * (4 * kLanes)) =
            __builtin_amdgcn_perm(sc[2 * j + 1], sc[2 * j], 0x06040200u);
      if constexpr (L::Wide) {
        // slot s (leaf s - 1) is row s
#pragma unroll
        for (int u = 0; u < Cap; ++u)
          *row(u + 1) = ((sc[u >> 1] >> (16 * (u & 1))) & 0xFF00u) | (uint32_t)u;
      } else {
#pragma unroll
        for (int r = 0; r < (Cap + 2) / 2; ++r) {
          // slot 2r: leaf 2r - 1 (count: byte 3 of sc[r - 1]); slot 2r + 1: leaf 2r (byte 1 of sc[r])
          const uint32_t lo = r > 0 ? (sc[r - 1] >> 16) & 0xFF00u : 0u;
          const uint32_t hi = r < Cap / 2 ? (sc[r] & 0xFF00u) << 16 : 0u;
          *row(r) = lo | hi | (uint32_t)(r > 0 ? 2 * r - 1 : 0) | (uint32_t)(2 * r) << 16;
        }
      }
    }

    // ---- heap, tree and codes (JPEG.c:913-983): the table is dead ------------
    bool over = tree_codes<Cap>(w, U, table + tile * kTablePerTile + bits_off(c), h0);

    // ---- encoded sequence, MSB-first (JPEG.c:993-1007) ------------------------
    uint8_t *const sout = bits + tile * kBitsPerTile + bits_off(c);
    constexpr int nwords = N / 2;                       // bits_cap / 32
    // A leaf's code word is its code left-aligned with its length in the low
    // 5 bits; the reads do not depend on the bit position, so each group of
    // kG positions' code words is read while the previous group is placed.
    // Each code is or-ed into the lane's zeroed bit rows at its bit position
    // (two ds_or: the word it starts in and the next), the rows past the code
    // table through the dead heap and symbols; two spill rows take the bits of
    // a stream that overflows its slot.  No exec branch per code: the
    // accumulator form stored each completed word under one.
    const LCol<uint32_t> codez{colp(&S.tab[L::ZeroRow][0])};
    constexpr int BitRow = L::CodeRow + Cap;
    static_assert(BitRow + nwords + 2 <= Keys / 4 + L::HeapRows + Cap / 4 &&
                      offsetof(L, heap) == sizeof(S.tab) && offsetof(L, sym) == offsetof(L, heap) + sizeof(S.heap),
                  "the bit rows fit the dead rows past the codes");
    uint8_t *const brow = reinterpret_cast<uint8_t *>(&S) + BitRow * (4 * kLanes) + 4 * lane;
    auto bit_row = [&](int r) { return reinterpret_cast<uint32_t *>(brow + r * (4 * kLanes)); };
    codez[0] = 0u;
#pragma unroll
    for (int r = 0; r < nwords + 2; ++r) *bit_row(r) = 0u;
    int pos = 0;
    constexpr int kG = 4;
    static_assert(N % kG == 0, "whole groups");
    auto ident = [&](int i, int h) {                    // leaf + 1 of emission h at position i, 0: none
      return (lid[i / 3] >> (10 * (i % 3) + 5 * h)) & 31u;
    };
    auto fetch = [&](int g, uint32_t (&cw)[2 * kG]) {
#pragma unroll
      for (int j = 0; j < 2 * kG; ++j) {
        cw[j] = codez[(int)ident(g * kG + j / 2, j & 1)];
      }
    };
    uint32_t cur[2 * kG], nxt[2 * kG];
    fetch(0, nxt);
#pragma unroll
    for (int g = 0; g < N / kG; ++g) {
#pragma unroll
      for (int j = 0; j < 2 * kG; ++j) cur[j] = nxt[j];
      if (g + 1 < N / kG) fetch(g + 1, nxt);
#pragma unroll
      for (int j = 0; j < 2 * kG; ++j) {
        const uint32_t al = cur[j] & ~31u;
        const uint32_t o = (uint32_t)pos & 31u;
        uint32_t *const r0 = bit_row(min(pos >> 5, nwords));
        atomicOr(r0, al >> o);
        atomicOr(r0 + kLanes, __builtin_amdgcn_alignbit(al, 0u, o));   // (o = 0: none)
        pos += (int)(cur[j] & 31u);
      }
    }
    const int nbits = pos;
    if (nbits > ref_bits_max(c)) over = true;           // char sequence[1024] / [512]
    // the slot's words, MSB-first bytes (16-B stores when the slot is aligned)
    {
      uint32_t wv[nwords];
#pragma unroll
      for (int r = 0; r < nwords; ++r) wv[r] = __builtin_bswap32(*bit_row(r));
      if ((reinterpret_cast<uintptr_t>(bits) & 15u) == 0) {
#pragma unroll
        for (int k = 0; k < nwords / 4; ++k)
          reinterpret_cast<uint4 *>(sout)[k] = make_uint4(wv[4 * k], wv[4 * k + 1], wv[4 * k + 2], wv[4 * k + 3]);
      } else {
#pragma unroll
        for (int r = 0; r < nwords; ++r) reinterpret_cast<uint32_t *>(sout)[r] = wv[r];
      }
    }
    meta[tile * 3 + c] = (uint32_t)(nbits < 0xFFFF ? nbits : 0xFFFF) | ((uint32_t)R << 16) |
                         ((uint32_t)U << 24);
    if constexpr (kLuma) {
      const uint64_t om = __ballot(over);
      if (lane == __builtin_ctzll(__ballot(1)))
        *lword = (uint32_t)__popcll(dm) | (uint32_t)__popcll(om) << 8;
    } else if (over) {
      atomicAdd(&status[0], 1u);
    }
  }
  if constexpr (!kLuma) {
    // Deferred streams (a symbol outside the table or more than Cap
    // distinct): the hashed encoder over this wave's LDS, which the fast path
    // has left dead -- the wave's own, then (an even wave) those of luma wave
    // lv, whose overflowed lanes it counts.  The dead LDS holds kSlots
    // working sets, so lanes 0 .. kSlots-1 each take every kSlots-th stream
    // of the list (a 4K image whose every luma stream defers: 15.97 ms with
    // one lane, 2.50 ms with 6; profiles/r06_ent_defer_defer_y.log).
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    constexpr int kSymO = 0, kHashO = kSymO + 2 * kFullCap, kHeapO = kHashO + 2 * kFullCap;
    constexpr int kCodeO = (kHeapO + 2 * (kFullCap + 2) + 3) & ~3, kLenO = kCodeO + 4 * kFullCap;
    constexpr int kStkO = (kLenO + kFullCap + 1) & ~1, kEnd = kStkO + 2 * (kFullCap + 1);
    constexpr int kSetB = (kEnd + 15) & ~15;                // one working set, 16-B aligned
    constexpr int kSlots = (int)sizeof(L) / kSetB < 8 ? (int)sizeof(L) / kSetB : 8;
    static_assert(kSlots >= 1, "the hashed encoder's arrays fit the wave's LDS");
    const uint32_t lw = (blockIdx.x & 1) ? 0u : *lword;
    const int nown = __popcll(dm), n = nown + (int)(lw & 255u);
    if (lane == 0 && (lw >> 8)) atomicAdd(&status[0], lw >> 8);
    // (the last wave's lanes past ntiles have returned: only live lanes take a share)
    const int nlive = (int)min((size_t)kLanes, ntiles - lv * kLanes);
    const int slots = kSlots < nlive ? kSlots : nlive;
    if (lane < slots && lane < n) {
      uint8_t *const lb = reinterpret_cast<uint8_t *>(&S) + lane * kSetB;
      const Work<GColT> ws{{reinterpret_cast<int16_t *>(lb + kSymO), 1}, {lb + kHashO, 1},
                           {reinterpret_cast<uint16_t *>(lb + kHeapO), 1},
                           {reinterpret_cast<uint32_t *>(lb + kCodeO), 1}, {lb + kLenO, 1},
                           {reinterpret_cast<uint16_t *>(lb + kStkO), 1}};
      uint64_t own = dm;                              // the wave's own deferred lanes, in order
      for (int j = 0; j < lane && own; ++j) own &= own - 1;
      for (int k = lane; k < n; k += slots) {
        uint32_t sid;                                 // tile * 3 + channel
        if (k < nown) {
          sid = (uint32_t)((lv * kLanes + __builtin_ctzll(own)) * 3 + c);
          for (int j = 0; j < slots && own; ++j) own &= own - 1;
        } else {
          sid = lst[k - nown];
        }
        const size_t t = sid / 3;
        const int cc = (int)(sid % 3);
        const int rc = encode_stream<kFullCap, 2 * kFullCap>(
            coef + t * 128 + coef_off(cc), stream_len(cc), ws,
            bits + t * kBitsPerTile + bits_off(cc), bits_cap(cc), ref_bits_max(cc),
            table + t * kTablePerTile + bits_off(cc), meta + t * 3 + cc);
        if (rc != kOk) atomicAdd(&status[0], 1u);
      }
    }
  }
}

// ---- decode ------------------------------------------------------------------

// Per stream up to 24 (luma) / 12 (chroma) codes, like the encoder's
// working set (more: regenerated per symbol, decode_stream_slow): the
// left-aligned codes in registers, each code's value and length in LDS as one
// u16 (value in 11 bits, two's complement, | length << 11: every value of a
// 4K image's streams fits; a stream whose values or lengths do not takes the
// slow path), one row of u16 per code.  With the decoded ints and the luma
// start map: 13.3 KiB per luma wave, 6.0 KiB per chroma wave (a lane decodes
// the tile's Cr, then its Cb stream), one of each per workgroup: a 4K image's
// 2,025 workgroups are all resident at once.
template <int N, int Cap>
struct DecLds {
  uint16_t vl[Cap][kLanes];                // code k: value | len << 11 (row k, the lane's u16)
  // the lane's decoded ints; rows of N + 2 (an odd number of dwords), so the
  // lanes' stores at one index hit 64 different banks (rows of N: 32-way)
  alignas(16) int16_t out[kLanes][N + 2];
  // luma: the lane's code starts as a 256-bit map over the 8-bit windows
  // (row r, bit 31 - i: window 32 r + i), for streams whose codes are all
  // <= 8 bits long
  uint32_t bm[N == 64 ? 8 : 1][kLanes];
};

// One lane's u16 column of a [rows][64] u16 block: entry k at byte k * 128
// (one address op per lookup; two lanes share a dword, so lanes reading
// different rows of the same bank pair conflict two-way at most)
struct VRow {
  typedef uint16_t __attribute__((may_alias)) HA;
  uint8_t *p;                                   // &block[0][lane] as bytes
  __device__ __forceinline__ HA &operator[](int k) const {
    return *reinterpret_cast<HA *>(p + (uint32_t)k * (2 * kLanes));
  }
};

// The number of k < Cap with h[k] > w (31-bit values): the borrows of
// w - h[k], taken by v_sub_co_u32 into SGPR pairs and summed by
// v_addc_co_u32 in two chains, eight codes per asm block (each carry is read
// at least eight instructions after its write: no hazard wait states; a
// group of four pads with an s_nop).
template <int Cap>
__device__ __forceinline__ uint32_t count_above(uint32_t w, const uint32_t (&h)[Cap]) {
  static_assert(Cap % 4 == 0, "groups of four");
  uint32_t a = 0, b = 0;
  if constexpr (Cap % 8 == 4) {
    uint32_t t0, t1, t2, t3;
    uint64_t c0, c1, c2, c3, d0, d1;
    asm("v_sub_co_u32_e64 %[t0], %[c0], %[w], %[h0]\n\t"
        "v_sub_co_u32_e64 %[t1], %[c1], %[w], %[h1]\n\t"
        "v_sub_co_u32_e64 %[t2], %[c2], %[w], %[h2]\n\t"
        "v_sub_co_u32_e64 %[t3], %[c3], %[w], %[h3]\n\t"
        "s_nop 1\n\t"
        "v_addc_co_u32_e64 %[a], %[d0], %[a], 0, %[c0]\n\t"
        "v_addc_co_u32_e64 %[b], %[d1], %[b], 0, %[c1]\n\t"
        "v_addc_co_u32_e64 %[a], %[d0], %[a], 0, %[c2]\n\t"
        "v_addc_co_u32_e64 %[b], %[d1], %[b], 0, %[c3]"
        : [a] "+v"(a), [b] "+v"(b), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2),
          [t3] "=&v"(t3), [c0] "=&s"(c0), [c1] "=&s"(c1), [c2] "=&s"(c2), [c3] "=&s"(c3),
          [d0] "=&s"(d0), [d1] "=&s"(d1)
        : [w] "v"(w), [h0] "v"(h[Cap - 4]), [h1] "v"(h[Cap - 3]), [h2] "v"(h[Cap - 2]),
          [h3] "v"(h[Cap - 1]));
  }
#pragma unroll
  for (int g = 0; g + 8 <= Cap; g += 8) {
    uint32_t t0, t1, t2, t3, t4, t5, t6, t7;
    uint64_t c0, c1, c2, c3, c4, c5, c6, c7, d0, d1;
    asm("v_sub_co_u32_e64 %[t0], %[c0], %[w], %[h0]\n\t"
        "v_sub_co_u32_e64 %[t1], %[c1], %[w], %[h1]\n\t"
        "v_sub_co_u32_e64 %[t2], %[c2], %[w], %[h2]\n\t"
        "v_sub_co_u32_e64 %[t3], %[c3], %[w], %[h3]\n\t"
        "v_sub_co_u32_e64 %[t4], %[c4], %[w], %[h4]\n\t"
        "v_sub_co_u32_e64 %[t5], %[c5], %[w], %[h5]\n\t"
        "v_sub_co_u32_e64 %[t6], %[c6], %[w], %[h6]\n\t"
        "v_sub_co_u32_e64 %[t7], %[c7], %[w], %[h7]\n\t"
        "v_addc_co_u32_e64 %[a], %[d0], %[a], 0, %[c0]\n\t"
        "v_addc_co_u32_e64 %[b], %[d1], %[b], 0, %[c1]\n\t"
        "v_addc_co_u32_e64 %[a], %[d0], %[a], 0, %[c2]\n\t"
        "v_addc_co_u32_e64 %[b], %[d1], %[b], 0, %[c3]\n\t"
        "v_addc_co_u32_e64 %[a], %[d0], %[a], 0, %[c4]\n\t"
        "v_addc_co_u32_e64 %[b], %[d1], %[b], 0, %[c5]\n\t"
        "v_addc_co_u32_e64 %[a], %[d0], %[a], 0, %[c6]\n\t"
        "v_addc_co_u32_e64 %[b], %[d1], %[b], 0, %[c7]"
        : [a] "+v"(a), [b] "+v"(b), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2),
          [t3] "=&v"(t3), [t4] "=&v"(t4), [t5] "=&v"(t5), [t6] "=&v"(t6), [t7] "=&v"(t7),
          [c0] "=&s"(c0), [c1] "=&s"(c1), [c2] "=&s"(c2), [c3] "=&s"(c3), [c4] "=&s"(c4),
          [c5] "=&s"(c5), [c6] "=&s"(c6), [c7] "=&s"(c7), [d0] "=&s"(d0), [d1] "=&s"(d1)
        : [w] "v"(w), [h0] "v"(h[g]), [h1] "v"(h[g + 1]), [h2] "v"(h[g + 2]),
          [h3] "v"(h[g + 3]), [h4] "v"(h[g + 4]), [h5] "v"(h[g + 5]), [h6] "v"(h[g + 6]),
          [h7] "v"(h[g + 7]));
  }
  return a + b;
}

// Decode one stream: bits + table -> RLE ints (decode_huffman) -> n ints
// (inverse_RLE: counts clamped to n, zero fill).  With one code (empty bit
// string) the reference decodes nothing and keeps its RLE ints: rle_len
// copies of the symbol.  tb: the table's first Cap entries; q0, q1: the
// first two 16-B chunks of the bits (loaded by the caller with the meta
// word); bm: the lane's start-map column (luma) or null.
// The symbol at a window is the count of codes <= it, minus one: the codes
// of a table built from a tree increase strictly (DFS order; a table whose
// codes do not is no tree and takes the slow path, which matches codes in
// table order).  When every code of the wave is <= 8 bits (a random 4K
// image's luma) the count is one row of a 256-bit map of the code starts
// plus that row's prefix count; otherwise Cap compares against the
// left-aligned codes in registers.  Only the matched entry's value | length
// is read from LDS (vl).
// The walk goes a (count, value) pair per step, so the inverse RLE's fill runs
// once per pair with every lane of the wave on it, and no lane carries a
// count across steps; the bit buffer is refilled once per one, two or four
// symbols, as the wave's longest code allows.  Every instruction of the walk
// counts: a wave issues at most one per four cycles, and two luma and two
// chroma waves share each SIMD.
// Returns 1 (decoded), 0 (malformed) or -1 (a value or length that the u16
// entries cannot hold, or codes that do not increase: the caller runs
// decode_stream_slow).
template <int Cap, typename VlT>
__device__ int decode_stream(const uint8_t *__restrict__ bits, uint32_t m,
                             const uint32_t (&tb)[Cap], uint4 q0, uint4 q1, VlT vl,
                             int16_t *__restrict__ out, int n, uint32_t *bm) {
  const int nbits = (int)(m & 0xFFFF), R = (int)((m >> 16) & 255), U = (int)(m >> 24);
  if (U == 0 || U > Cap || R == 0 || R > 2 * n) return 0;
  // codes from the lengths, left to right (DFS order); lh[k] = lc[k] >> 1 (a
  // code of <= 31 bits leaves bit 0 of its left-aligned form clear), all ones
  // past U: above every 31-bit window, never counted as <= it
  uint32_t lh[Cap];
  uint32_t code = 0, prev = 0;
  int plen = 0, lmax = 0;
  bool bad = false, wide = false;
#pragma unroll
  for (int k = 0; k < Cap; ++k) {
    lh[k] = ~0u;
    if (k < U) {
      const uint32_t e = tb[k];
      const int L = (int)((e >> 16) & 255);
      const int v = (int16_t)(e & 0xFFFF);
      bad = bad || L > 32 || (U > 1 && L == 0);
      wide = wide || L > 31 || v < -1024 || v > 1023;
      if (k) code = L >= plen ? (code + 1) << (L - plen) : (code + 1) >> (plen - L);
      plen = L;
      lmax = max(lmax, L);
      const uint32_t lc = L ? code << (32 - L) : 0;
      wide = wide || (k && lc <= prev);
      prev = lc;
      lh[k] = lc >> 1;
      vl[k] = (uint16_t)(((uint32_t)v & 0x7FFu) | ((uint32_t)L << 11));
    }
  }
  if (bad) return 0;
  if (wide) return -1;
  int idx = 0;
  // a run of cnt copies of v at idx (clamped to the row): the first store
  // unconditionally (past the run it is overwritten by the next run or the
  // final zero fill; the row has spare slots), a loop only for longer runs
  // (an empty asm keeps the loop a loop: as a memset it compiled to three
  // nested loops whose exec-mask bookkeeping every pair paid)
  auto fill = [&](int cnt, int v) {
    const int c = min(cnt, n - idx);
    out[idx] = (int16_t)v;
    for (int j = 1; j < c; ++j) {
      out[idx + j] = (int16_t)v;
      asm volatile("");
    }
    idx += max(c, 0);
  };
  // an entry's value (11-bit two's complement) and length
  auto val = [](uint32_t e) { return (int)((int32_t)(e << 21) >> 21); };
  if (U == 1) {
    const int v = val(vl[0]);
    for (int j = 0; j + 1 < R; j += 2) fill(v, v);
  } else {
    // MSB-first bit buffer: acc holds nacc valid bits, left-aligned; words
    // come from 16-B chunks of the stream's slot, the next chunk in flight.
    // Chunks past the bits are read too (they lie in the slot, and what they
    // hold cannot change a decode: see lookup), so the load needs no select.
    const uint4 *src = reinterpret_cast<const uint4 *>(bits);
    const int last = n / 8 - 1;                       // the slot's last chunk
    uint4 q = q0, nxt = q1;
    int qi = 0, ci = 1;
    uint64_t acc = 0;
    int nacc = 0, p = 0, got = 0;
    // s codes lie above the window, a suffix of the increasing codes: the
    // entry is k = Cap - 1 - s, at byte -128 s from entry Cap - 1
    const uint8_t *vbase = reinterpret_cast<const uint8_t *>(&vl[Cap - 1]);
    // Codes of at most 8 bits in every stream of the wave: the symbol at a
    // window is found from its top 8 bits as the count of code starts <= them
    // -- one row of the lane's 256-bit start map (LDS, built with ors) and
    // that row's prefix count (registers, a byte each) instead of Cap
    // compares.  Wave-uniform, so no lane walks both.
    const bool narrow = __ballot(lmax > 8) == 0;      // every code <= 8 bits
    const bool mid = __ballot(lmax > 16) == 0;        // every code <= 16 bits
    const bool use_bm = bm != nullptr && narrow;
    uint32_t pa = 0, pb = 0;
    if (use_bm) {
#pragma unroll
      for (int r = 0; r < 8; ++r) bm[r * kLanes] = 0u;
#pragma unroll
      for (int k = 0; k < Cap; ++k)
        if (k < U) {
          const uint32_t st = lh[k] >> 23;       // the code's top 8 bits
          atomicOr(&bm[(st >> 5) * kLanes], 0x80000000u >> (st & 31));
        }
      uint32_t run = 0;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        if (r < 4) pa |= run << (8 * r);
        else pb |= run << (8 * (r - 4));
        run += __builtin_popcount(bm[r * kLanes]);
      }
    }
    auto refill = [&]() {
      if (nacc <= 32) {                               // refill 32 bits (codes <= 31)
        // the chunk's words move down as they are used (an indexed select
        // became a scratch array)
        const uint32_t wd = q.x;
        q.x = q.y;
        q.y = q.z;
        q.z = q.w;
        acc |= (uint64_t)__builtin_bswap32(wd) << (32 - nacc);
        nacc += 32;
        if (++qi == 4) {
          qi = 0;
          q = nxt;
          ci = ci < last ? ci + 1 : ci;
          nxt = src[ci];
        }
      }
    };
    auto lookup = [&]() -> uint32_t {
      // 32 bits at p.  Bits past the end are not masked: the codes increase
      // strictly, so they are prefix-free, and a code that fits in the bits
      // left is found whatever follows them (one that does not fit is
      // malformed either way)
      const uint32_t win = (uint32_t)(acc >> 32);
      if (use_bm) {
        const uint32_t w8 = win >> 24, j = w8 >> 5;
        const uint32_t row = bm[j * kLanes];
        const uint32_t before = __builtin_amdgcn_perm(pb, pa, j | 0x0C0C0C00u);
        const int cnt = (int)(__builtin_popcount(row >> (31 - (w8 & 31))) + before);
        return vl[cnt - 1];
      }
      // borrows of win - lh[k] in two carry chains through SGPR pairs (the
      // compare-and-add form serialised every code on VCC)
      const uint32_t above = count_above<Cap>(win >> 1, lh);
      return *reinterpret_cast<const uint16_t *>(vbase - (int)(above * (2 * kLanes)));
    };
    // one symbol at p (bits in acc): its entry; a code past the end ends the
    // walk as malformed (flagged, no branch out of the loop per symbol)
    auto take = [&](bool &bd) -> uint32_t {
      const uint32_t e = lookup();
      const int L = (int)(e >> 11);
      bd = p + L > nbits;
      bad = bad || bd;
      p = bd ? nbits : p + L;
      acc <<= L;
      nacc -= L;
      ++got;
      return e;
    };
    // a (count, value) pair: the count, then (bits left) its value and the run
    auto pair = [&](bool refill_each) {
      if (refill_each) refill();
      bool b0, b1;
      const uint32_t e0 = take(b0);
      if (p < nbits) {
        if (refill_each) refill();
        const uint32_t e1 = take(b1);
        if (!b1) fill(val(e0), val(e1));
      }
    };
    // a refill leaves >= 33 bits: four symbols when every code of the wave
    // is <= 8 bits, two when <= 16, else one (wave-uniform cadence)
    if (narrow) {
      while (p < nbits) {
        refill();
        pair(false);
        if (p < nbits) pair(false);
      }
    } else if (mid) {
      while (p < nbits) {
        refill();
        pair(false);
      }
    } else {
      while (p < nbits) pair(true);
    }
    if (bad || got != R) return 0;
  }
  while (idx < n) out[idx++] = 0;
  return 1;
}

// Streams with more codes than the LDS table holds (> 24 luma / 12 chroma:
// the encoder's deferred streams): the codes are regenerated from the table
// for every symbol and searched linearly -- slow, rare, no storage.
__device__ bool decode_stream_slow(const uint8_t *__restrict__ bits, uint32_t m,
                                   const uint32_t *__restrict__ table, int16_t *__restrict__ out,
                                   int n) {
  const int nbits = (int)(m & 0xFFFF), R = (int)((m >> 16) & 255), U = (int)(m >> 24);
  if (R == 0 || R > 2 * n) return false;
  const uint32_t *wds = reinterpret_cast<const uint32_t *>(bits);
  int p = 0, got = 0, idx = 0, pending = -1;
  while (p < nbits) {
    const int wi = p >> 5, sh = p & 31;
    const uint32_t w0 = __builtin_bswap32(wds[wi]);
    const uint32_t w1 = (wi + 1) * 32 < nbits ? __builtin_bswap32(wds[wi + 1]) : 0;
    uint32_t win = sh ? (w0 << sh) | (w1 >> (32 - sh)) : w0;
    if (nbits - p < 32) win &= ~0u << (32 - (nbits - p));
    uint32_t code = 0;
    int plen = 0, hit = -1, L = 0;
    for (int k = 0; k < U && hit < 0; ++k) {
      L = (int)((table[k] >> 16) & 255);
      if (L == 0 || L > 32) return false;
      if (k) code = L >= plen ? (code + 1) << (L - plen) : (code + 1) >> (plen - L);
      plen = L;
      if ((win >> (32 - L)) == code) hit = k;
    }
    if (hit < 0 || p + L > nbits) return false;
    const int v = (int16_t)(table[hit] & 0xFFFF);
    if (pending < 0) {
      pending = v;
    } else {
      int cnt = pending;
      pending = -1;
      if (idx + cnt > n) cnt = n - idx;
      for (int j = 0; j < cnt; ++j) out[idx++] = (int16_t)v;
    }
    p += L;
    ++got;
  }
  if (got != R) return false;
  while (idx < n) out[idx++] = 0;
  return true;
}

// One wave's 64 tiles of one channel group: luma (a lane decodes its tile's
// Y stream) or chroma (its Cr, then its Cb stream).
template <bool kLuma>
__device__ __forceinline__ void decode_wave(DecLds<kLuma ? 64 : 32, kLuma ? kFastCap : kChromaCap> &S,
                                            int lane, size_t group,
                                            const uint8_t *__restrict__ bits,
                                            const uint32_t *__restrict__ meta,
                                            const uint32_t *__restrict__ table, size_t ntiles,
                                            int16_t *__restrict__ coef,
                                            uint32_t *__restrict__ status, uint32_t tag) {
  constexpr int Cap = kLuma ? kFastCap : kChromaCap;
  const size_t tile = group * kLanes + lane;
  if (tile >= ntiles) return;
  uint32_t fails = 0;
  // ints are produced one at a time: collect them in LDS, then 16-B stores
  // (2-byte stores to 64 scattered streams wrote ~6x the bytes)
  int16_t *o = S.out[lane];
  const VRow vl{reinterpret_cast<uint8_t *>(&S.vl[0][lane])};
#pragma unroll 1
  for (int c = kLuma ? 0 : 1; c <= (kLuma ? 0 : 2); ++c) {
    const uint32_t m = meta[tile * 3 + c];
    const uint8_t *b = bits + tile * kBitsPerTile + bits_off(c);
    const uint32_t *t = table + tile * kTablePerTile + bits_off(c);
    // the table's first Cap entries and the first two 16-B chunks of the
    // bits, loaded with the meta word (all inside the stream's slots, whatever
    // the meta word says): one wait, where a load per code under its k < U
    // test was waited for code by code
    uint32_t tb[Cap];
#pragma unroll
    for (int i = 0; i < Cap / 4; ++i) {
      const uint4 v = reinterpret_cast<const uint4 *>(t)[i];
      tb[4 * i] = v.x;
      tb[4 * i + 1] = v.y;
      tb[4 * i + 2] = v.z;
      tb[4 * i + 3] = v.w;
    }
    const uint4 q0 = reinterpret_cast<const uint4 *>(b)[0];
    const uint4 q1 = reinterpret_cast<const uint4 *>(b)[1];
    const int U = (int)(m >> 24);
    const int n = stream_len(c);
    // a foreign or corrupted meta word must not index past the stream's
    // slot: its bits (bits_cap bits) and its table (2 n entries: RLE of n ints)
    const bool sane = (int)(m & 0xFFFF) <= bits_cap(c) && U <= 2 * n;
    bool ok = false;
    if (!sane)  // a use on this path too, so the loads are not sunk past the meta test
      asm volatile("" ::"v"(tb[0]), "v"(q0.x), "v"(q1.x));
    if (sane) {
      const int r = U <= Cap ? decode_stream<Cap>(b, m, tb, q0, q1, vl, o, n,
                                                   kLuma ? &S.bm[0][lane] : nullptr)
                             : -1;
      ok = r < 0 ? decode_stream_slow(b, m, t, o, n) : r != 0;
    } else {
      for (int j = 0; j < n; ++j) o[j] = 0;
    }
    fails += !ok;
    uint4 *dst = reinterpret_cast<uint4 *>(coef + tile * 128 + coef_off(c));
    const uint32_t *src = reinterpret_cast<const uint32_t *>(o);    // 4-B aligned rows
    for (int v = 0; v < n / 8; ++v)
      dst[v] = make_uint4(src[4 * v], src[4 * v + 1], src[4 * v + 2], src[4 * v + 3]);
  }
  // the wave's malformed streams, added to status[1] once workgroup 0 has
  // zeroed it for this call (status[2] = the call's tag; see the kernel)
  const uint32_t f = (uint32_t)__popcll(__ballot(fails & 1)) + 2u * (uint32_t)__popcll(__ballot(fails & 2));
  if (f && lane == __builtin_ctzll(__ballot(1))) {
    for (int spin = 0; spin < (1 << 22) &&
                       __hip_atomic_load(&status[2], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != tag;
         ++spin)
      __builtin_amdgcn_s_sleep(2);
    atomicAdd(&status[1], f);
  }
}

// A workgroup is two waves over the same 64 tiles: wave 0 decodes their luma
// streams, wave 1 their chroma streams, each in its own LDS (12 + 6.4 KB: a
// 4K image's 2,025 workgroups are all resident at once, a luma and a chroma
// wave beside each other on every SIMD).  One launch: the luma and chroma
// kernels side by side on two streams started the chroma waves 8 us late and
// paid the fork and join.
// status[1] is zeroed here, not by a memset ahead of the launch (a dispatch
// and its gap): workgroup 0, dispatched first and waiting on nothing, zeroes
// it and then publishes the call's tag in status[2]; a wave with malformed
// streams adds them only once it reads that tag (bounded spin), so no add
// can precede the zero.
__global__ __launch_bounds__(2 * kLanes) void entropy_decode_kernel(
    const uint8_t *__restrict__ bits, const uint32_t *__restrict__ meta,
    const uint32_t *__restrict__ table, size_t ntiles, int16_t *__restrict__ coef,
    uint32_t *__restrict__ status, uint32_t tag) {
  __shared__ DecLds<64, kFastCap> SY;
  __shared__ DecLds<32, kChromaCap> SC;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    status[1] = 0u;
    __threadfence();
    __hip_atomic_store(&status[2], tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int lane = threadIdx.x & (kLanes - 1);
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) < kLanes)
    decode_wave<true>(SY, lane, blockIdx.x, bits, meta, table, ntiles, coef, status, tag);
  else
    decode_wave<false>(SC, lane, blockIdx.x, bits, meta, table, ntiles, coef, status, tag);
}

// one tag per decode call (status[2]); 0 is skipped, so a zeroed status
// never matches
std::atomic<uint32_t> g_decode_tag{0};

}  // namespace

// the luma waves' deferred lists and words (the scratch layout above)
extern "C" size_t jpegr_entropy_scratch_bytes(size_t ntiles) {
  return (ntiles + kLanes - 1) / kLanes * (kLanes + 1) * sizeof(uint32_t);
}

extern "C" int jpegr_entropy_encode_device(const void *d_coef, size_t ntiles, void *d_bits,
                                           void *d_meta, void *d_table, void *d_scratch,
                                           void *d_status, void *stream) {
  if (!d_coef || !d_bits || !d_meta || !d_table || !d_scratch || !d_status || ntiles == 0 ||
      ntiles > ((size_t)1 << 32) / 3 || (reinterpret_cast<uintptr_t>(d_coef) & 15) != 0 ||
      (reinterpret_cast<uintptr_t>(d_bits) & 3) != 0)
    return JPEGR_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  auto *lists = static_cast<uint32_t *>(d_scratch);
  auto *status = static_cast<uint32_t *>(d_status);
  const unsigned groups = (unsigned)((ntiles + kLanes - 1) / kLanes);
  // (one stream: side by side, as the decoder runs, measured 0.140 -> 0.146 ms
  // per 4K image -- the encoder's luma and chroma waves contend for the same
  // LDS and issue slots, and the fork / join costs more than it overlaps)
  hipLaunchKernelGGL(entropy_encode_lane<true>, dim3(groups), dim3(kLanes), 0, s,
                     static_cast<const int16_t *>(d_coef), ntiles, static_cast<uint8_t *>(d_bits),
                     static_cast<uint32_t *>(d_meta), static_cast<uint32_t *>(d_table), lists,
                     status);
  hipLaunchKernelGGL(entropy_encode_lane<false>, dim3(groups * 2), dim3(kLanes), 0, s,
                     static_cast<const int16_t *>(d_coef), ntiles, static_cast<uint8_t *>(d_bits),
                     static_cast<uint32_t *>(d_meta), static_cast<uint32_t *>(d_table), lists,
                     status);
  return hipGetLastError() == hipSuccess ? JPEGR_OK : JPEGR_ERR_HIP;
}

extern "C" int jpegr_entropy_decode_device(const void *d_bits, const void *d_meta,
                                           const void *d_table, size_t ntiles, void *d_coef,
                                           void *d_status, void *stream) {
  if (!d_bits || !d_meta || !d_table || !d_coef || !d_status || ntiles == 0 ||
      ntiles > ((size_t)1 << 32) / 3 || (reinterpret_cast<uintptr_t>(d_coef) & 15) != 0 ||
      (reinterpret_cast<uintptr_t>(d_bits) & 15) != 0 ||
      (reinterpret_cast<uintptr_t>(d_table) & 15) != 0 ||
      (reinterpret_cast<uintptr_t>(d_status) & 3) != 0)
    return JPEGR_ERR_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t tag = ++g_decode_tag;
  if (tag == 0) tag = ++g_decode_tag;
  const unsigned groups = (unsigned)((ntiles + kLanes - 1) / kLanes);
  hipLaunchKernelGGL(entropy_decode_kernel, dim3(groups), dim3(2 * kLanes), 0, s,
                     static_cast<const uint8_t *>(d_bits), static_cast<const uint32_t *>(d_meta),
                     static_cast<const uint32_t *>(d_table), ntiles, static_cast<int16_t *>(d_coef),
                     static_cast<uint32_t *>(d_status), tag);
  return hipGetLastError() == hipSuccess ? JPEGR_OK : JPEGR_ERR_HIP;
}

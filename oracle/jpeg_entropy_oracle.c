/*
 * oracle/jpeg_entropy_oracle.c -- TEST INFRASTRUCTURE ONLY (CPU checker).
 *
 * Plain-C restatement of the reference's JPEG entropy stage for one stream
 * (the zigzagged ints of one channel of one tile), Algorithms/sequential/
 * JPEG/JPEG.c:
 *   RLE                    :767-808   (count, value) ints, (int) comparisons
 *   calculate_frequency    :864-886   symbols = int + 1000, first-occurrence order
 *   heapify / build_heap   :895-936   min-heap on count, strict <, left before right
 *   build_huffman_tree     :938-962   pop, pop, append the merged node and call
 *                                     heapify on its (leaf) index -- a no-op, so
 *                                     the new node is NOT sifted up
 *   assign_codes           :964-983   DFS, left '0', right '1', codes[] in DFS order
 *   generate_encoded_sequence :993-1007  concatenated codes
 *   decode_huffman / inverse_RLE :1009-1033, :810-840
 * Output layout (the GPU kernel's): codes as (value, length,
 * bits) in the reference's codes[] order; the '0'/'1' string packed MSB-first.
 * Pinned against the reference's own functions by tests/test_oracle.py
 * (oracle/ref_jpeg_harness.c: ref_jpeg_entropy).  Only tests/ and bench's
 * cpu_baseline leg load this.
 */
#include <stdint.h>
#include <string.h>

#define JE_MAXSYM 128           /* RLE of 64 ints: <= 128 ints */
#define JE_MAXNODE (2 * JE_MAXSYM)

typedef struct {
  int count, value, left, right;   /* value -1 = internal (JPEG.c:952) */
} je_node;

static void je_heapify(const je_node *nodes, int *heap, int size, int i)   /* JPEG.c:895 */
{
  for (;;) {
    int smallest = i, l = 2 * i + 1, r = 2 * i + 2;
    if (l < size && nodes[heap[l]].count < nodes[heap[smallest]].count) smallest = l;
    if (r < size && nodes[heap[r]].count < nodes[heap[smallest]].count) smallest = r;
    if (smallest == i) return;
    int t = heap[i];
    heap[i] = heap[smallest];
    heap[smallest] = t;
    i = smallest;
  }
}

typedef struct {
  int16_t *val;
  uint8_t *len;
  uint64_t *code;
  int n;
  int overflow;                 /* a code longer than 63 bits */
} je_codes;

static void je_assign(const je_node *nodes, int id, uint64_t code, int depth, je_codes *c)
{                                                                /* JPEG.c:964 */
  const je_node *nd = &nodes[id];
  if (nd->value != -1) {
    c->val[c->n] = (int16_t)(nd->value - 1000);
    c->len[c->n] = (uint8_t)depth;
    c->code[c->n] = code;
    c->n++;
    return;
  }
  if (depth >= 63) {
    c->overflow = 1;
    return;
  }
  je_assign(nodes, nd->left, code << 1, depth + 1, c);
  je_assign(nodes, nd->right, (code << 1) | 1, depth + 1, c);
}

/*
 * One stream of n (<= 64) ints.  Outputs: rle[<=128] and *rle_len; the code
 * table in DFS order: *ncodes entries of (tab_val, tab_len, tab_code, the
 * code's bits right-aligned); the encoded bits packed MSB-first into bits
 * (cap_bits bits of room) and *nbits.  Returns 0, or -1 if a code is longer
 * than 63 bits or the bits do not fit cap_bits (the reference's fixed
 * buffers would overflow long before: char code[32], char sequence[1024]).
 */
int jo_entropy_stream(const int16_t *zz, int n, int *rle, int *rle_len, int *ncodes,
                      int16_t *tab_val, uint8_t *tab_len, uint64_t *tab_code, uint8_t *bits,
                      int cap_bits, int *nbits)
{
  /* RLE (JPEG.c:767-808): values are exact ints, so (int) comparisons are == */
  int R = 0, cur = zz[0], cnt = 1;
  for (int i = 1; i <= n; i++) {
    if (i < n && zz[i] == cur) {
      cnt++;
    } else {
      rle[R++] = cnt;
      rle[R++] = cur;
      if (i < n) {
        cur = zz[i];
        cnt = 1;
      }
    }
  }
  *rle_len = R;

  /* frequencies, first-occurrence order (JPEG.c:864-886) */
  je_node nodes[JE_MAXNODE];
  int U = 0;
  for (int j = 0; j < R; j++) {
    const int s = rle[j] + 1000;
    int u = 0;
    while (u < U && nodes[u].value != s) u++;
    if (u == U) {
      nodes[U].value = s;
      nodes[U].count = 0;
      nodes[U].left = nodes[U].right = -1;
      U++;
    }
    nodes[u].count++;
  }

  /* heap of node ids (JPEG.c:913-936), tree (JPEG.c:938-962) */
  int heap[JE_MAXSYM];
  for (int i = 0; i < U; i++) heap[i] = i;
  for (int i = U / 2 - 1; i >= 0; i--) je_heapify(nodes, heap, U, i);
  int size = U, next = U;
  while (size > 1) {
    const int left = heap[0];
    heap[0] = heap[--size];
    je_heapify(nodes, heap, size, 0);
    const int right = heap[0];
    heap[0] = heap[--size];
    je_heapify(nodes, heap, size, 0);
    nodes[next].count = nodes[left].count + nodes[right].count;
    nodes[next].value = -1;
    nodes[next].left = left;
    nodes[next].right = right;
    heap[size++] = next++;
    je_heapify(nodes, heap, size, size - 1);     /* a leaf: no-op, as in the reference */
  }

  je_codes c = {tab_val, tab_len, tab_code, 0, 0};
  je_assign(nodes, heap[0], 0, 0, &c);
  *ncodes = c.n;
  if (c.overflow) return -1;

  /* encoded sequence (JPEG.c:993-1007): codes looked up by symbol */
  int nb = 0;
  memset(bits, 0, (size_t)(cap_bits + 7) / 8);
  for (int j = 0; j < R; j++) {
    int k = 0;
    while (tab_val[k] != rle[j]) k++;
    const int L = tab_len[k];
    if (nb + L > cap_bits) return -1;
    for (int t = L - 1; t >= 0; t--, nb++)
      if ((tab_code[k] >> t) & 1) bits[nb >> 3] |= (uint8_t)(0x80 >> (nb & 7));
  }
  *nbits = nb;
  return 0;
}

/*
 * Decode side: bits + code table (DFS order) -> RLE ints (decode_huffman,
 * JPEG.c:1009-1033; with a one-symbol table, whose code is empty, the
 * reference decodes nothing and keeps its RLE array: rle_len copies of the
 * symbol) -> n ints (inverse_RLE, JPEG.c:810-840, clamped to n, zero-filled).
 */
int jo_entropy_decode(const uint8_t *bits, int nbits, int rle_len, int ncodes,
                      const int16_t *tab_val, const uint8_t *tab_len, const uint64_t *tab_code,
                      int n, int16_t *zz)
{
  int rle[JE_MAXSYM];
  int R = 0;
  if (ncodes == 1) {
    for (R = 0; R < rle_len && R < JE_MAXSYM; R++) rle[R] = tab_val[0];
  } else {
    int p = 0;
    while (p < nbits && R < JE_MAXSYM) {
      int k = -1;
      for (int c = 0; c < ncodes && k < 0; c++) {
        const int L = tab_len[c];
        if (p + L > nbits) continue;
        uint64_t v = 0;
        for (int t = 0; t < L; t++) v = (v << 1) | ((bits[(p + t) >> 3] >> (7 - ((p + t) & 7))) & 1);
        if (v == tab_code[c]) k = c;
      }
      if (k < 0) return -1;
      rle[R++] = tab_val[k];
      p += tab_len[k];
    }
  }
  int idx = 0;
  for (int i = 0; i + 1 < R; i += 2) {
    int count = rle[i];
    if (idx + count > n) count = n - idx;
    for (int j = 0; j < count; j++) zz[idx++] = (int16_t)rle[i + 1];
  }
  while (idx < n) zz[idx++] = 0;
  return 0;
}

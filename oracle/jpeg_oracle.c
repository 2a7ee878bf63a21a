/*
 * oracle/jpeg_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference JPEG hot path: RGB->Y/Cr/Cb, 4:2:2 odd-
 * column subsampling, 8x8 / 8x4 tiling, naive fp64 DCT-II, truncating
 * quantisation and zigzag.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product never does.
 *
 * Must be compiled as strict IEEE binary64 with no contraction
 * (-O2 -ffp-contract=off, no -march=native): the parity target is the
 * sequential C compiled for x86-64 SSE2.
 *
 * Parity pin: checked against the reference's own JPEG.c compiled from its
 * sources (oracle/ref_jpeg_harness.c -> oracle/_ref/) and against the
 * SURVEY.md Appendix A4 md5s and 8x8 literal KAT (tests/test_oracle.py).
 *
 * Output layout (defined by this build; the reference keeps doubles in
 * memory): per tile, int16 little-endian [Y 64 zigzag][Cr 32 zigzag]
 * [Cb 32 zigzag]; tiles in raster order.  Pixels outside the image are 0
 * (divide_image zero-initialises, JPEG.c:512-523).
 *
 * Citations are to /root/reference/Algorithms/sequential/JPEG/JPEG.c.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

#define JO_PI 3.14159265358979323846                         /* JPEG.c:11 */

static const size_t JO_LUMA_Q[64] = {                          /* JPEG.c:12 */
    8, 6, 6, 8, 10, 14, 18, 22,   6, 6, 7, 9, 12, 20, 22, 20,
    6, 7, 8, 10, 14, 22, 25, 22,  8, 9, 10, 14, 18, 28, 27, 22,
    10, 12, 14, 18, 22, 35, 33, 26, 14, 18, 22, 22, 27, 33, 36, 30,
    18, 22, 26, 28, 33, 40, 40, 34, 22, 26, 28, 30, 36, 34, 35, 33};
static const size_t JO_CHROMA_Q[32] = {                        /* JPEG.c:22 */
    17, 18, 24, 47, 18, 21, 26, 66, 24, 26, 56, 99, 47, 66, 99, 99,
    66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

static uint8_t jo_clamp(int v)                                  /* JPEG.c:132 */
{
    if (v < 0) return 0;
    if (v > 255) return 255;
    return (uint8_t)v;
}

/* JPEG.c:127 */
static uint8_t jo_luma(unsigned r, unsigned g, unsigned b)
{
    double y = 0.299 * r + 0.587 * g + 0.114 * b;
    return (uint8_t)y;
}
/* JPEG.c:157 */
static uint8_t jo_cr(unsigned r, unsigned g, unsigned b)
{
    return jo_clamp((int)(0.439 * r - 0.368 * g - 0.071 * b + 128));
}
/* JPEG.c:180 */
static uint8_t jo_cb(unsigned r, unsigned g, unsigned b)
{
    return jo_clamp((int)(-0.148 * r - 0.291 * g + 0.439 * b + 128));
}

/* discrete_cosine_transform, JPEG.c:451-494 (width = columns, height = rows)
 * The cos() arguments are exactly the reference expression; values are
 * tabulated once because cos is a pure function of them. */
void jo_dct(const uint8_t *data, size_t width, size_t height, double *coef)
{
    double cx[8][8], cy[8][8];
    for (size_t x = 0; x < height; x++)
        for (size_t u = 0; u < height; u++)
            cx[x][u] = cos((JO_PI * (2 * x + 1) * u) / (2.0 * height)); /* :481 */
    for (size_t y = 0; y < width; y++)
        for (size_t v = 0; v < width; v++)
            cy[y][v] = cos((JO_PI * (2 * y + 1) * v) / (2.0 * width));  /* :482 */
    int cv[64];
    for (size_t i = 0; i < width * height; i++)
        cv[i] = (int)data[i] - 128;                                   /* :467 */
    for (size_t u = 0; u < height; u++) {
        for (size_t v = 0; v < width; v++) {
            double sum = 0.0;
            for (size_t x = 0; x < height; x++)
                for (size_t y = 0; y < width; y++)
                    sum += cv[x * width + y] * cx[x][u] * cy[y][v];   /* :483 */
            double au = (u == 0) ? sqrt(1.0 / height) : sqrt(2.0 / height);
            double av = (v == 0) ? sqrt(1.0 / width) : sqrt(2.0 / width);
            coef[u * width + v] = au * av * sum;                      /* :489 */
        }
    }
}

/* Quantize, JPEG.c:621-629 */
void jo_quantize(double *c, const size_t *table, size_t size)
{
    for (size_t i = 0; i < size; i++) {
        c[i] /= table[i];
        c[i] = (int)c[i];
    }
}

/* zigzag_pattern, JPEG.c:693-728 */
void jo_zigzag(size_t width, size_t height, const double *in, double *out)
{
    size_t index = 0;
    for (size_t sum = 0; sum < width + height - 1; sum++) {
        size_t start_row = (sum < width) ? 0 : sum - width + 1;
        size_t end_row = (sum < height) ? sum : height - 1;
        if (sum % 2 == 0) {
            for (size_t row = end_row; row >= start_row && row < height; row--) {
                size_t col = sum - row;
                if (col < width) out[index++] = in[row * width + col];
            }
        } else {
            for (size_t row = start_row; row <= end_row; row++) {
                size_t col = sum - row;
                if (col < width) out[index++] = in[row * width + col];
            }
        }
    }
}

/* Gather one tile's planes (divide_image JPEG.c:496-550 after
 * chroma_subsample JPEG.c:302-375: chroma sample c' of a tile comes from
 * pixel column 8*bc + 2*c' + 1). */
static void jo_tile_inputs(const uint8_t *rgba, int w, int h, int br, int bc,
                           uint8_t ylum[64], uint8_t cr[32], uint8_t cb[32])
{
    memset(ylum, 0, 64);
    memset(cr, 0, 32);
    memset(cb, 0, 32);
    int cs_w = w / 2;                                  /* chroma_subsample :314 */
    for (int r = 0; r < 8; r++) {
        int row = 8 * br + r;
        if (row >= h) break;
        for (int c = 0; c < 8; c++) {
            int col = 8 * bc + c;
            if (col >= w) break;
            const uint8_t *px = rgba + ((size_t)row * w + col) * 4;
            ylum[r * 8 + c] = jo_luma(px[0], px[1], px[2]);
            if ((c % 2) == 0) {                        /* divide_image :540 */
                int k = col / 2;                       /* index into Cs row */
                uint8_t vr = 0, vb = 0;
                if (k < cs_w) {
                    const uint8_t *q = rgba + ((size_t)row * w + 2 * k + 1) * 4;
                    vr = jo_cr(q[0], q[1], q[2]);
                    vb = jo_cb(q[0], q[1], q[2]);
                }
                cr[r * 4 + c / 2] = vr;
                cb[r * 4 + c / 2] = vb;
            }
        }
    }
}

/* One tile -> 128 int16 coefficients [Y64 zz][Cr32 zz][Cb32 zz]. */
void jo_encode_tile(const uint8_t *rgba, int w, int h, int br, int bc,
                    int16_t *out)
{
    uint8_t ylum[64], cr[32], cb[32];
    double c[64], z[64];
    jo_tile_inputs(rgba, w, h, br, bc, ylum, cr, cb);
    jo_dct(ylum, 8, 8, c);                                    /* JPEG.c:1138 */
    jo_quantize(c, JO_LUMA_Q, 64);                             /* JPEG.c:1146 */
    jo_zigzag(8, 8, c, z);                                     /* JPEG.c:1176 */
    for (int i = 0; i < 64; i++) out[i] = (int16_t)z[i];
    jo_dct(cr, 4, 8, c);                                       /* JPEG.c:1139 */
    jo_quantize(c, JO_CHROMA_Q, 32);                           /* JPEG.c:1148 */
    jo_zigzag(4, 8, c, z);                                     /* JPEG.c:1177 */
    for (int i = 0; i < 32; i++) out[64 + i] = (int16_t)z[i];
    jo_dct(cb, 4, 8, c);                                       /* JPEG.c:1140 */
    jo_quantize(c, JO_CHROMA_Q, 32);                           /* JPEG.c:1147 */
    jo_zigzag(4, 8, c, z);                                     /* JPEG.c:1178 */
    for (int i = 0; i < 32; i++) out[96 + i] = (int16_t)z[i];
}

/* Un-quantised fp64 DCT coefficients of one tile, row-major (not zigzag):
 * [Y 64][Cr 32][Cb 32] doubles.  Used to check the GPU's raw DCT bit-exactly. */
void jo_dct_tile_raw(const uint8_t *rgba, int w, int h, int br, int bc,
                     double *out)
{
    uint8_t ylum[64], cr[32], cb[32];
    jo_tile_inputs(rgba, w, h, br, bc, ylum, cr, cb);
    jo_dct(ylum, 8, 8, out);
    jo_dct(cr, 4, 8, out + 64);
    jo_dct(cb, 4, 8, out + 96);
}

int jo_tiles_x(int w) { return (w + 7) / 8; }
int jo_tiles_y(int h) { return (h + 7) / 8; }

/* Whole image, tile rows [ty0, ty1). */
void jo_encode_rows(const uint8_t *rgba, int w, int h, int ty0, int ty1,
                    int16_t *out)
{
    int tx = jo_tiles_x(w);
    for (int br = ty0; br < ty1; br++)
        for (int bc = 0; bc < tx; bc++)
            jo_encode_tile(rgba, w, h, br, bc,
                           out + ((size_t)br * tx + bc) * 128);
}

void jo_encode_image(const uint8_t *rgba, int w, int h, int16_t *out)
{
    jo_encode_rows(rgba, w, h, 0, jo_tiles_y(h), out);
}

void jo_dct_raw_image(const uint8_t *rgba, int w, int h, double *out)
{
    int tx = jo_tiles_x(w), ty = jo_tiles_y(h);
    for (int br = 0; br < ty; br++)
        for (int bc = 0; bc < tx; bc++)
            jo_dct_tile_raw(rgba, w, h, br, bc,
                            out + ((size_t)br * tx + bc) * 128);
}

/* Y/Cr/Cb planes (build_*_matrix), for colour-conversion parity. */
void jo_planes(const uint8_t *rgba, int w, int h, uint8_t *Y, uint8_t *Cr,
               uint8_t *Cb)
{
    for (size_t i = 0; i < (size_t)w * h; i++) {
        const uint8_t *p = rgba + 4 * i;
        Y[i] = jo_luma(p[0], p[1], p[2]);
        Cr[i] = jo_cr(p[0], p[1], p[2]);
        Cb[i] = jo_cb(p[0], p[1], p[2]);
    }
}

/* ---- multi-threaded CPU baseline ------------------------------------- */
typedef struct {
    const uint8_t *rgba;
    int w, h, ty0, ty1;
    int16_t *out;
} jo_job;

static void *jo_worker(void *a)
{
    jo_job *j = (jo_job *)a;
    jo_encode_rows(j->rgba, j->w, j->h, j->ty0, j->ty1, j->out);
    return NULL;
}

void jo_encode_image_parallel(const uint8_t *rgba, int w, int h, int threads,
                              int16_t *out)
{
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    int ty = jo_tiles_y(h);
    pthread_t tid[256];
    jo_job jobs[256];
    int per = (ty + threads - 1) / threads;
    for (int t = 0; t < threads; t++) {
        int a = t * per, b = a + per;
        if (a > ty) a = ty;
        if (b > ty) b = ty;
        jobs[t] = (jo_job){rgba, w, h, a, b, out};
        pthread_create(&tid[t], NULL, jo_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
}

/* glibc rand() seeded stream as in random_image.c:64-73 (rand() is never
 * seeded there, i.e. seed 1): per pixel r,g,b = rand()%256, a = 255. */
void jo_rand_image(unsigned seed, int w, int h, uint8_t *rgba)
{
    srand(seed);
    for (size_t i = 0; i < (size_t)w * h; i++) {
        rgba[4 * i + 0] = (uint8_t)(rand() % 256);
        rgba[4 * i + 1] = (uint8_t)(rand() % 256);
        rgba[4 * i + 2] = (uint8_t)(rand() % 256);
        rgba[4 * i + 3] = 255;
    }
}

/* ---- reconstruction (the decode side of the reference's main) ----------- */

/* inverse_discrete_cosine_transform, JPEG.c:399-448: for x < H, y < W,
 * sum over u (outer) and v (inner) of ((((au*av)*c)*cos_x)*cos_y), then
 * (int)round(sum + 128) clamped to [0, 255]. */
void jo_idct(const double *coef, size_t width, size_t height, uint8_t *values)
{
    double cx[8][8], cy[8][8];
    for (size_t x = 0; x < height; x++)
        for (size_t u = 0; u < height; u++)
            cx[x][u] = cos((JO_PI * (2 * x + 1) * u) / (2.0 * height)); /* :425 */
    for (size_t y = 0; y < width; y++)
        for (size_t v = 0; v < width; v++)
            cy[y][v] = cos((JO_PI * (2 * y + 1) * v) / (2.0 * width));  /* :426 */
    for (size_t x = 0; x < height; x++)
        for (size_t y = 0; y < width; y++) {
            double sum = 0.0;
            for (size_t u = 0; u < height; u++)
                for (size_t v = 0; v < width; v++) {
                    double au = (u == 0) ? sqrt(1.0 / height) : sqrt(2.0 / height);
                    double av = (v == 0) ? sqrt(1.0 / width) : sqrt(2.0 / width);
                    sum += au * av * coef[u * width + v] * cx[x][u] * cy[y][v];  /* :428 */
                }
            int value = (int)round(sum + 128.0);                        /* :440 */
            values[x * width + y] = value < 0 ? 0 : (value > 255 ? 255 : (uint8_t)value);
        }
}

/* zigzag positions of a width x height block: pos[k] = natural index of
 * zigzag element k (jo_zigzag's order; reverse_zigzag_pattern, JPEG.c:729-764,
 * visits the same cells in the same order) */
static void jo_zigzag_pos(size_t width, size_t height, int *pos)
{
    double nat[64], zz[64];
    for (size_t i = 0; i < width * height; i++) nat[i] = (double)i;
    jo_zigzag(width, height, nat, zz);
    for (size_t k = 0; k < width * height; k++) pos[k] = (int)zz[k];
}

/* One tile's reconstructed samples from its 128 zigzag int16 coefficients:
 * reverse zigzag, Inverse_quantize (JPEG.c:631-638), IDCT. */
void jo_decode_tile(const int16_t *coef, uint8_t ylum[64], uint8_t cr[32], uint8_t cb[32])
{
    int p8[64], p4[32];
    jo_zigzag_pos(8, 8, p8);
    jo_zigzag_pos(4, 8, p4);
    double c[64];
    for (int k = 0; k < 64; k++) c[p8[k]] = (double)coef[k];
    for (int i = 0; i < 64; i++) c[i] *= JO_LUMA_Q[i];
    jo_idct(c, 8, 8, ylum);
    for (int k = 0; k < 32; k++) c[p4[k]] = (double)coef[64 + k];
    for (int i = 0; i < 32; i++) c[i] *= JO_CHROMA_Q[i];
    jo_idct(c, 4, 8, cr);
    for (int k = 0; k < 32; k++) c[p4[k]] = (double)coef[96 + k];
    for (int i = 0; i < 32; i++) c[i] *= JO_CHROMA_Q[i];
    jo_idct(c, 4, 8, cb);
}

/* reconstructed.png pixels (JPEG.c:1131-1425): tiles below
 * ceil(W*H/64) are decoded; the rest keep their original tile samples (the
 * reference never transforms them, :1131, but assemble_image walks every
 * tile); assemble_image (JPEG.c:553-619) converts YCbCr 4:2:2 to RGB. */
void jo_reconstruct_image(const uint8_t *rgba, int w, int h, uint8_t *out)
{
    const int tx = jo_tiles_x(w), ty = jo_tiles_y(h);
    const size_t total_blocks = ((size_t)w * h + 63) / 64;
    for (int br = 0; br < ty; br++)
        for (int bc = 0; bc < tx; bc++) {
            const size_t i = (size_t)br * tx + bc;
            uint8_t yl[64], cr[32], cb[32];
            if (i < total_blocks) {
                int16_t q[128];
                jo_encode_tile(rgba, w, h, br, bc, q);
                jo_decode_tile(q, yl, cr, cb);
            } else {
                jo_tile_inputs(rgba, w, h, br, bc, yl, cr, cb);
            }
            for (int r = 0; r < 8; r++)
                for (int c = 0; c < 8; c++) {
                    const int row = 8 * br + r, col = 8 * bc + c;
                    if (row >= h || col >= w) continue;
                    const int Y = yl[r * 8 + c];
                    const int Cb = cb[r * 4 + c / 2], Cr = cr[r * 4 + c / 2];
                    int R = Y + (int)(1.402 * (Cr - 128));                 /* :601 */
                    int G = Y - (int)(0.344136 * (Cb - 128)) - (int)(0.714136 * (Cr - 128));
                    int B = Y + (int)(1.772 * (Cb - 128));
                    uint8_t *o = out + ((size_t)row * w + col) * 4;
                    o[0] = jo_clamp(R);
                    o[1] = jo_clamp(G);
                    o[2] = jo_clamp(B);
                    o[3] = 255;
                }
        }
}

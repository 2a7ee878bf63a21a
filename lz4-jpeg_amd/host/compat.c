/*
 * compat.c -- the reference's function-level API (include/lz4jpeg_compat.h)
 * on top of the MI355X C ABI.  Host C: file handling, buffer moves and the
 * reference's exit(1) error behaviour; every byte of compression / DCT /
 * quantisation / zigzag is computed by the HIP kernels.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/jpegr.h"
#include "../../include/lz4jpeg_compat.h"
#include "../../include/lz4r.h"
#include "lzj_host.h"

/* safe_open, LZ4.c:109-120 */
static FILE *safe_open(const char *name, const char *mode) {
  FILE *f = fopen(name, mode);
  if (f == NULL) {
    perror("Error: Unable to open file");
    exit(1);
  }
  return f;
}

static uint8_t *read_all(FILE *f, size_t *n) {
  if (fseek(f, 0, SEEK_END) != 0) return NULL;
  long sz = ftell(f);
  if (sz < 0 || fseek(f, 0, SEEK_SET) != 0) return NULL;
  uint8_t *b = (uint8_t *)malloc((size_t)sz + 1);
  if (!b) return NULL;
  *n = fread(b, 1, (size_t)sz, f);
  return b;
}

/* dump_to_hex_file, LZ4.c:75-107: every byte as "%02X " */
static void dump_to_hex_file(const char *in_name, const char *out_name) {
  FILE *in = fopen(in_name, "rb");
  if (!in) {
    perror("Error opening input file");
    return;
  }
  FILE *out = fopen(out_name, "w");
  if (!out) {
    perror("Error opening output file");
    fclose(in);
    return;
  }
  int c;
  while ((c = fgetc(in)) != EOF) fprintf(out, "%02X ", (unsigned)c);
  fclose(in);
  fclose(out);
}

static void die_hip(const char *what, int rc) {
  fprintf(stderr, "Error: %s failed (%d)\n", what, rc);
  exit(1);
}

void lz4_encode(void) {
  FILE *log_file = safe_open(LZ4_LOG_FILE, "a");
  FILE *input_file = safe_open(LZ4_INPUT_FILE, "r");
  FILE *output_file = safe_open(LZ4_COMPRESSED_FILE, "ab");
  size_t n = 0;
  uint8_t *data = read_all(input_file, &n);
  fclose(input_file);
  if (!data) {
    perror("Error: Failed to read input file");
    exit(1);
  }
  if (n < LZ4R_BLOCK) {                                   /* LZ4.c:632-637 */
    printf("Error: default block length is too high, please reduce it before proceding.");
    exit(1);
  }
  const size_t cap = lz4r_compress_bound(n);
  uint8_t *comp = (uint8_t *)malloc(cap);
  size_t got = 0;
  if (!comp) {
    perror("Error: Unable to allocate memory");
    exit(1);
  }
  int rc = lz4r_compress(data, n, comp, cap, &got);
  if (rc != LZ4R_OK) die_hip("lz4r_compress", rc);
  if (fwrite(comp, 1, got, output_file) != got) {
    perror("Error: write failed");
    exit(1);
  }
  fclose(log_file);
  fclose(output_file);
  free(comp);
  free(data);
  dump_to_hex_file(LZ4_COMPRESSED_FILE, LZ4_HEX_FILE);
}

/* ---- the match provider of the per-block API (host/compat_lz4.c) ---------
 * Every position's len | dist << 16 of the n-byte block at `in`, from one
 * launch: lz4r_block_matches_device for a 300-byte (or shorter) block,
 * lz4r_window_matches_device (the reference's whole 65535-byte window,
 * MAX_MATCH_LENGTH 1024) for a longer block_length.  Device buffers grow to
 * the block; per thread. */
static __thread struct {
  size_t cap;
  void *d_in, *d_match;
} fm_dev;

int lzj_block_matches(const uint8_t *in, size_t n, uint32_t *match) {
  if (n > fm_dev.cap) {
    (void)hipFree(fm_dev.d_in);
    (void)hipFree(fm_dev.d_match);
    fm_dev.d_in = fm_dev.d_match = NULL;
    fm_dev.cap = 0;
    /* +16: the block kernel's staging may read a few bytes past a short block */
    if (hipMalloc(&fm_dev.d_in, n + 16) != hipSuccess ||
        hipMalloc(&fm_dev.d_match, n * sizeof(uint32_t)) != hipSuccess)
      return LZ4R_ERR_NOMEM;
    fm_dev.cap = n;
  }
  if (hipMemcpy(fm_dev.d_in, in, n, hipMemcpyHostToDevice) != hipSuccess) return LZ4R_ERR_HIP;
  const int rc = n <= LZ4R_BLOCK ? lz4r_block_matches_device(fm_dev.d_in, n, fm_dev.d_match, NULL)
                                 : lz4r_window_matches_device(fm_dev.d_in, n, fm_dev.d_match, NULL);
  if (rc != LZ4R_OK) return rc;
  if (hipMemcpy(match, fm_dev.d_match, n * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
    return LZ4R_ERR_HIP;
  return LZ4R_OK;
}

void LZ4_decode(char *input_bin_file, char *log) {
  FILE *input_file = safe_open(input_bin_file, "rb");
  FILE *log_file = safe_open(log, "a");
  size_t n = 0;
  uint8_t *comp = read_all(input_file, &n);
  fclose(input_file);
  fclose(log_file);
  if (!comp) {
    perror("Error: Failed to read input file");
    exit(1);
  }
  /* every block decodes to at most 300 bytes and takes at least 8 */
  size_t cap = (n / 8 + 1) * LZ4R_BLOCK;
  uint8_t *out = (uint8_t *)malloc(cap);
  size_t got = 0;
  if (!out) {
    perror("Error: Unable to allocate memory");
    exit(1);
  }
  /* on the GPU: block boundaries found on the device from the stream alone */
  int rc = lz4r_decompress_stream(comp, n, out, cap, &got);
  if (rc != LZ4R_OK) {
    fprintf(stderr, "Error: %s\n", lz4r_strerror(rc));
    exit(1);
  }
  FILE *f = safe_open(LZ4_UNCOMPRESSED_FILE, "w");
  if (fwrite(out, 1, got, f) != got) {
    perror("Error: write failed");
    exit(1);
  }
  fclose(f);
  free(out);
  free(comp);
}

/* ---- JPEG: one block per call, on the GPU --------------------------------- */

static void *dmalloc(size_t n) {
  void *p = NULL;
  if (hipMalloc(&p, n) != hipSuccess) {
    fprintf(stderr, "Memory allocation failed!\n");
    exit(EXIT_FAILURE);
  }
  return p;
}

void discrete_cosine_transform(uint8_t *data, size_t width, size_t height,
                               double **coefficients) {
  const size_t n = width * height;
  *coefficients = (double *)malloc(n * sizeof(double));
  if (!*coefficients) {
    fprintf(stderr, "Memory allocation failed!\n");
    exit(EXIT_FAILURE);
  }
  uint8_t *din = (uint8_t *)dmalloc(n);
  double *dout = (double *)dmalloc(n * sizeof(double));
  int rc = hipMemcpy(din, data, n, hipMemcpyHostToDevice) == hipSuccess ? JPEGR_OK
                                                                          : JPEGR_ERR_HIP;
  if (rc == JPEGR_OK) rc = jpegr_dct_blocks_device(din, (int)width, (int)height, 1, dout, NULL);
  if (rc == JPEGR_OK &&
      hipMemcpy(*coefficients, dout, n * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  (void)hipFree(din);
  (void)hipFree(dout);
  if (rc != JPEGR_OK) die_hip("jpegr_dct_blocks_device", rc);
}

void Quantize(double **luminance, size_t *table, size_t size) {
  double *tab = (double *)malloc(size * sizeof(double));
  if (!tab) {
    fprintf(stderr, "Memory allocation failed!\n");
    exit(EXIT_FAILURE);
  }
  for (size_t i = 0; i < size; ++i) tab[i] = (double)table[i];     /* JPEG.c:626 */
  double *dc = (double *)dmalloc(size * sizeof(double));
  double *dt = (double *)dmalloc(size * sizeof(double));
  int rc = JPEGR_OK;
  if (hipMemcpy(dc, *luminance, size * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dt, tab, size * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  if (rc == JPEGR_OK) rc = jpegr_quantize_device(dc, dt, (int)size, size, NULL);
  if (rc == JPEGR_OK &&
      hipMemcpy(*luminance, dc, size * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  (void)hipFree(dc);
  (void)hipFree(dt);
  free(tab);
  if (rc != JPEGR_OK) die_hip("jpegr_quantize_device", rc);
}

/* Scan order of zigzag_pattern (JPEG.c:693-728): diagonals sum = row + col,
 * even sums bottom-to-top, odd sums top-to-bottom.  perm[k] = source index. */
static size_t zigzag_order(size_t width, size_t height, int *perm) {
  size_t k = 0;
  for (size_t sum = 0; sum + 1 < width + height; ++sum) {
    const size_t r0 = sum < width ? 0 : sum - width + 1;
    const size_t r1 = sum < height ? sum : height - 1;
    if (sum % 2 == 0) {
      for (size_t row = r1 + 1; row-- > r0;)
        if (sum - row < width) perm[k++] = (int)(row * width + (sum - row));
    } else {
      for (size_t row = r0; row <= r1; ++row)
        if (sum - row < width) perm[k++] = (int)(row * width + (sum - row));
    }
  }
  return k;
}

void zigzag_pattern(size_t width, size_t height, double *input, double *output) {
  const size_t n = width * height;
  int *perm = (int *)malloc(n * sizeof(int));
  if (!perm) {
    fprintf(stderr, "Memory allocation failed!\n");
    exit(EXIT_FAILURE);
  }
  const size_t k = zigzag_order(width, height, perm);
  double *din = (double *)dmalloc(n * sizeof(double));
  double *dout = (double *)dmalloc(n * sizeof(double));
  int *dperm = (int *)dmalloc(n * sizeof(int));
  int rc = JPEGR_OK;
  if (hipMemcpy(din, input, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dperm, perm, n * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  if (rc == JPEGR_OK && k > 0) rc = jpegr_permute_device(din, dout, dperm, (int)k, k, NULL);
  if (rc == JPEGR_OK &&
      hipMemcpy(output, dout, k * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = JPEGR_ERR_HIP;
  (void)hipFree(din);
  (void)hipFree(dout);
  (void)hipFree(dperm);
  free(perm);
  if (rc != JPEGR_OK) die_hip("jpegr_permute_device", rc);
}

/*
 * JPEG_seq / JPEG_par -- drop-ins for the reference's JPEG_seq.exe
 * (Algorithms/sequential/JPEG/JPEG.c main, :1099-1460) and JPEG_par.exe
 * (spawned by Experiment/JPEG_parallel_experiment.c:99 system("JPEG_par.exe");
 * the committed JPEG_par.exe reads and writes the same files as JPEG_seq.exe
 * and computes the same tiles, one Win32 thread per 8x8 block) on the MI355X
 * path: one program, installed under both names.
 *
 * File contract (run from Experiment/, JPEG_sequential_experiment.c:99):
 *   reads  ../Assets/Images/rand_8X8.png            (JPEG.c:9, :1102)
 *   writes ../Output-Input/Images/original.png, luminance.png,
 *          rChrominance.png, bChrominance.png       (JPEG.c:1105, :1121-1123)
 *          ../Output-Input/Images/reconstructed.png (JPEG.c:1408-1428)
 *          ../Output-Input/Images/coefficients.bin  the quantised zigzag
 *          coefficients: int16 LE per 8x8 tile [Y 64][Cr 32][Cb 32], tiles
 *          in raster order (the reference keeps them in memory only)
 *   exit 0; unreadable image: "Error loading image" and exit(1) (JPEG.c:74-78).
 * Colour planes, DCT, quantisation, zigzag, the entropy round trip the
 * reference runs per tile (RLE + Huffman encode, decode, inverse RLE,
 * JPEG.c:1211-1349) and the reconstruction (reverse zigzag, dequantisation,
 * IDCT, YCbCr->RGB) run on the GPU (jpegr_*); reconstructed.png is decoded
 * from the entropy-decoded coefficients, as in the reference.
 * Optional argv[1] / argv[2] override the input image / output directory.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/jpegr.h"
#include "lzj_host.h"

#define IMAGES_DIRECTORY "../Assets/Images/"
#define OUTPUT_DIRECTORY "../Output-Input/Images/"

static void fail(const char *what) {
  fprintf(stderr, "Error: %s\n", what);
  exit(1);
}

static void write_png(const char *dir, const char *name, int w, int h, const uint8_t *rgba) {
  char path[4096];
  snprintf(path, sizeof path, "%s%s", dir, name);
  if (lzj_png_write(path, w, h, rgba) != 0) printf("Error: Failed to write the PNG image.\n");
}

/* (uint8_t) of the reference's double expression: gcc/x86-64 truncates to
 * int, then keeps the low byte (JPEG.c:234-236, 263-266, 288-291). */
static uint8_t u8_of(double v) { return (uint8_t)(int)v; }

int main(int argc, char **argv) {
  const char *in_path = argc > 1 ? argv[1] : IMAGES_DIRECTORY "rand_8X8.png";
  const char *out_dir = argc > 2 ? argv[2] : OUTPUT_DIRECTORY;
  int w = 0, h = 0;
  uint8_t *rgba = NULL;
  if (lzj_png_read(in_path, &w, &h, &rgba) != 0) {
    printf("Error loading image\n");
    exit(1);
  }
  const size_t npx = (size_t)w * h;
  const size_t ncoef = jpegr_coef_count(w, h);
  const size_t ntiles = ncoef / 128;
  void *d_rgba = NULL, *d_y = NULL, *d_cr = NULL, *d_cb = NULL, *d_coef = NULL, *d_rec = NULL;
  void *d_bits = NULL, *d_meta = NULL, *d_table = NULL, *d_scr = NULL, *d_st = NULL;
  void *d_coef2 = NULL;
  if (hipMalloc(&d_rgba, npx * 4) != hipSuccess || hipMalloc(&d_y, npx) != hipSuccess ||
      hipMalloc(&d_rec, npx * 4) != hipSuccess ||
      hipMalloc(&d_cr, npx) != hipSuccess || hipMalloc(&d_cb, npx) != hipSuccess ||
      hipMalloc(&d_coef, ncoef * 2) != hipSuccess || hipMalloc(&d_coef2, ncoef * 2) != hipSuccess ||
      hipMalloc(&d_bits, ntiles * 256) != hipSuccess ||
      hipMalloc(&d_meta, ntiles * 3 * 4) != hipSuccess ||
      hipMalloc(&d_table, ntiles * 256 * 4) != hipSuccess ||
      hipMalloc(&d_scr, jpegr_entropy_scratch_bytes(ntiles)) != hipSuccess ||
      hipMalloc(&d_st, 16) != hipSuccess ||
      hipMemset(d_st, 0, 16) != hipSuccess)
    fail("device allocation failed");
  if (hipMemcpy(d_rgba, rgba, npx * 4, hipMemcpyHostToDevice) != hipSuccess) fail("copy in");
  if (jpegr_planes_device(d_rgba, w, h, d_y, d_cr, d_cb, NULL) != JPEGR_OK ||
      jpegr_encode_device(d_rgba, w, h, 1, d_coef, NULL) != JPEGR_OK ||
      jpegr_entropy_encode_device(d_coef, ntiles, d_bits, d_meta, d_table, d_scr, d_st, NULL) !=
          JPEGR_OK ||
      jpegr_entropy_decode_device(d_bits, d_meta, d_table, ntiles, d_coef2, d_st, NULL) !=
          JPEGR_OK ||
      jpegr_reconstruct_device(d_coef2, d_rgba, w, h, 1, d_rec, NULL) != JPEGR_OK)
    fail("kernel launch");
  uint32_t st[2];
  if (hipMemcpy(st, d_st, 8, hipMemcpyDeviceToHost) != hipSuccess) fail("copy out");
  if (st[1] != 0) fail("entropy decode");
  uint8_t *y = malloc(npx), *cr = malloc(npx), *cb = malloc(npx), *vis = malloc(npx * 4);
  uint8_t *rec = malloc(npx * 4);
  int16_t *coef = malloc(ncoef * 2);
  if (!y || !cr || !cb || !vis || !coef || !rec) fail("out of memory");
  if (hipMemcpy(y, d_y, npx, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(cr, d_cr, npx, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(cb, d_cb, npx, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(coef, d_coef, ncoef * 2, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(rec, d_rec, npx * 4, hipMemcpyDeviceToHost) != hipSuccess)
    fail("copy out");

  write_png(out_dir, "original.png", w, h, rgba);                    /* JPEG.c:1105 */
  for (size_t i = 0; i < npx; ++i) {                                   /* JPEG.c:218-241 */
    vis[4 * i] = vis[4 * i + 1] = vis[4 * i + 2] = y[i];
    vis[4 * i + 3] = 255;
  }
  write_png(out_dir, "luminance.png", w, h, vis);
  for (size_t i = 0; i < npx; ++i) {                                   /* JPEG.c:253-276 */
    vis[4 * i] = u8_of(128 + 1.402 * (cr[i] - 128));
    vis[4 * i + 1] = u8_of(128 - 0.344 * (128 - 128) - 0.714 * (cr[i] - 128));
    vis[4 * i + 2] = u8_of(128 + 1.772 * (128 - 128));
    vis[4 * i + 3] = 255;
  }
  write_png(out_dir, "rChrominance.png", w, h, vis);
  for (size_t i = 0; i < npx; ++i) {                                   /* JPEG.c:278-300 */
    vis[4 * i] = u8_of(128 + 1.402 * (128 - 128));
    vis[4 * i + 1] = u8_of(128 - 0.344 * (cb[i] - 128) - 0.714 * (128 - 128));
    vis[4 * i + 2] = u8_of(128 + 1.772 * (cb[i] - 128));
    vis[4 * i + 3] = 255;
  }
  write_png(out_dir, "bChrominance.png", w, h, vis);
  write_png(out_dir, "reconstructed.png", w, h, rec);                 /* JPEG.c:1428 */

  char path[4096];
  snprintf(path, sizeof path, "%scoefficients.bin", out_dir);
  FILE *f = fopen(path, "wb");
  if (!f || fwrite(coef, 2, ncoef, f) != ncoef) fail("cannot write coefficients.bin");
  fclose(f);
  (void)hipFree(d_rgba); (void)hipFree(d_y); (void)hipFree(d_cr); (void)hipFree(d_cb);
  (void)hipFree(d_coef); (void)hipFree(d_rec); (void)hipFree(d_coef2); (void)hipFree(d_bits);
  (void)hipFree(d_meta); (void)hipFree(d_table); (void)hipFree(d_scr); (void)hipFree(d_st);
  free(rgba); free(y); free(cr); free(cb); free(vis); free(coef); free(rec);
  return 0;
}

/*
 * oracle/ref_jpeg_harness.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Compiles the reference's own sequential JPEG.c, unmodified and where it
 * lies (REF_JPEG_C, passed by oracle/Makefile), with its main() renamed, and
 * drives its hot-path functions in-process so the C restatement in
 * jpeg_oracle.c can be pinned against the real thing.  Output goes only to
 * oracle/_ref/ (git-ignored).  Nothing here is copied from the reference:
 * the reference source is #included from /root/reference at build time.
 *
 * Exposed: ref_jpeg_encode_image(rgba, w, h, out) producing the same int16
 * layout as jo_encode_image ([Y64 zz][Cr32 zz][Cb32 zz] per tile, raster),
 * following the reference's main loop JPEG.c:1110-1178.
 */
#define main ref_jpeg_main
#include REF_JPEG_C
#undef main

int ref_jpeg_encode_image(const unsigned char *rgba, int w, int h,
                          short *out)
{
    ImageData img;
    img.width = w;
    img.height = h;
    img.pixel_count = (size_t)w * h;
    img.pixels = malloc(h * sizeof(Pixel *));
    for (int y = 0; y < h; y++) {
        img.pixels[y] = malloc(w * sizeof(Pixel));
        for (int x = 0; x < w; x++) {
            const unsigned char *p = rgba + ((size_t)y * w + x) * 4;
            img.pixels[y][x].r = p[0];
            img.pixels[y][x].g = p[1];
            img.pixels[y][x].b = p[2];
            img.pixels[y][x].a = p[3];
        }
    }
    uint8_t **lum, **cr, **cb;
    build_luminance_matrix(img, &lum);          /* JPEG.c:1111 */
    build_rChrominance_matrix(img, &cr);        /* JPEG.c:1115 */
    build_bChrominance_matrix(img, &cb);        /* JPEG.c:1119 */
    chroma_subsample(&cb, img);                 /* JPEG.c:1126 */
    chroma_subsample(&cr, img);                 /* JPEG.c:1129 */
    size_t tx = (w + 7) / 8, ty = (h + 7) / 8;
    PixelGroup *blocks = divide_image(lum, cr, cb, img, 8);   /* :1133 */
    for (size_t i = 0; i < tx * ty; i++) {
        discrete_cosine_transform(blocks[i].lum_values, 8, 8,
                                  &blocks[i].lum_coefficients);
        discrete_cosine_transform(blocks[i].r_values, 4, 8,
                                  &blocks[i].r_coefficients);
        discrete_cosine_transform(blocks[i].b_values, 4, 8,
                                  &blocks[i].b_coefficients);
        Quantize(&blocks[i].lum_coefficients, LUMINANCE_QUANTIZATION_TABLE, 64);
        Quantize(&blocks[i].b_coefficients, CHROMINANCE_QUANTIZATION_TABLE, 32);
        Quantize(&blocks[i].r_coefficients, CHROMINANCE_QUANTIZATION_TABLE, 32);
        double zl[64], zr[32], zb[32];
        zigzag_pattern(8, 8, blocks[i].lum_coefficients, zl);
        zigzag_pattern(4, 8, blocks[i].r_coefficients, zr);
        zigzag_pattern(4, 8, blocks[i].b_coefficients, zb);
        short *o = out + i * 128;
        for (int k = 0; k < 64; k++) o[k] = (short)zl[k];
        for (int k = 0; k < 32; k++) o[64 + k] = (short)zr[k];
        for (int k = 0; k < 32; k++) o[96 + k] = (short)zb[k];
        free(blocks[i].lum_coefficients);
        free(blocks[i].r_coefficients);
        free(blocks[i].b_coefficients);
    }
    free(blocks);
    for (int y = 0; y < h; y++) { free(lum[y]); free(cr[y]); free(cb[y]); }
    free(lum); free(cr); free(cb);
    free_pixels(img.pixels, h);
    return 0;
}

/* Raw (un-quantised) DCT doubles of every tile, row-major per plane. */
int ref_jpeg_dct_raw(const unsigned char *rgba, int w, int h, double *out)
{
    ImageData img;
    img.width = w;
    img.height = h;
    img.pixel_count = (size_t)w * h;
    img.pixels = malloc(h * sizeof(Pixel *));
    for (int y = 0; y < h; y++) {
        img.pixels[y] = malloc(w * sizeof(Pixel));
        for (int x = 0; x < w; x++) {
            const unsigned char *p = rgba + ((size_t)y * w + x) * 4;
            img.pixels[y][x].r = p[0];
            img.pixels[y][x].g = p[1];
            img.pixels[y][x].b = p[2];
            img.pixels[y][x].a = p[3];
        }
    }
    uint8_t **lum, **cr, **cb;
    build_luminance_matrix(img, &lum);
    build_rChrominance_matrix(img, &cr);
    build_bChrominance_matrix(img, &cb);
    chroma_subsample(&cb, img);
    chroma_subsample(&cr, img);
    size_t tx = (w + 7) / 8, ty = (h + 7) / 8;
    PixelGroup *blocks = divide_image(lum, cr, cb, img, 8);
    for (size_t i = 0; i < tx * ty; i++) {
        double *c;
        discrete_cosine_transform(blocks[i].lum_values, 8, 8, &c);
        memcpy(out + i * 128, c, 64 * sizeof(double));
        free(c);
        discrete_cosine_transform(blocks[i].r_values, 4, 8, &c);
        memcpy(out + i * 128 + 64, c, 32 * sizeof(double));
        free(c);
        discrete_cosine_transform(blocks[i].b_values, 4, 8, &c);
        memcpy(out + i * 128 + 96, c, 32 * sizeof(double));
        free(c);
    }
    free(blocks);
    for (int y = 0; y < h; y++) { free(lum[y]); free(cr[y]); free(cb[y]); }
    free(lum); free(cr); free(cb);
    free_pixels(img.pixels, h);
    return 0;
}

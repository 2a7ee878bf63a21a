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

/* The reference's whole per-block pipeline after the DCT, as its main()
 * runs it (JPEG.c:1131-1423): Quantize, zigzag, RLE, the per-block Huffman
 * encode -> decode round trip, inverse RLE, reverse zigzag,
 * Inverse_quantize, IDCT for the first ceil(W*H/64) blocks, then
 * assemble_image over every tile.  out_rgba receives the pixels main()
 * writes to reconstructed.png. */
int ref_jpeg_reconstruct(const unsigned char *rgba, int w, int h, unsigned char *out_rgba)
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
    size_t total_blocks = (size_t)ceil((double)img.pixel_count / 64);      /* :1131 */
    PixelGroup *blocks = divide_image(lum, cr, cb, img, 8);
    for (size_t i = 0; i < total_blocks; i++) {                              /* :1136-1149 */
        discrete_cosine_transform(blocks[i].lum_values, 8, 8, &blocks[i].lum_coefficients);
        discrete_cosine_transform(blocks[i].r_values, 4, 8, &blocks[i].r_coefficients);
        discrete_cosine_transform(blocks[i].b_values, 4, 8, &blocks[i].b_coefficients);
        Quantize(&blocks[i].lum_coefficients, LUMINANCE_QUANTIZATION_TABLE, 64);
        Quantize(&blocks[i].b_coefficients, CHROMINANCE_QUANTIZATION_TABLE, 32);
        Quantize(&blocks[i].r_coefficients, CHROMINANCE_QUANTIZATION_TABLE, 32);
    }
    for (size_t i = 0; i < total_blocks; i++) {                              /* :1159-1405 */
        double tl[64], tr[32], tb[32];
        zigzag_pattern(8, 8, blocks[i].lum_coefficients, tl);
        zigzag_pattern(4, 8, blocks[i].r_coefficients, tr);
        zigzag_pattern(4, 8, blocks[i].b_coefficients, tb);
        for (size_t j = 0; j < 64; j++) blocks[i].lum_coefficients[j] = tl[j];
        for (size_t j = 0; j < 32; j++) {
            blocks[i].r_coefficients[j] = tr[j];
            blocks[i].b_coefficients[j] = tb[j];
        }
        size_t ll, lr, lb;
        RLE(tl, 64, &blocks[i].RLE_encoded_lum, &ll);
        RLE(tr, 32, &blocks[i].RLE_encoded_r, &lr);
        RLE(tb, 32, &blocks[i].RLE_encoded_b, &lb);
        int *enc[3] = {blocks[i].RLE_encoded_lum, blocks[i].RLE_encoded_r, blocks[i].RLE_encoded_b};
        size_t el[3] = {ll, lr, lb};
        for (int c = 0; c < 3; c++) {
            size_t ncode;
            Node *root;
            HuffmanCode *codes = encode_huffman(enc[c], el[c], &ncode, &root);
            char seq[2048];
            generate_encoded_sequence(enc[c], el[c], codes, ncode, seq);
            size_t dl;
            double *dec = decode_huffman(root, seq, &dl);
            for (size_t j = 0; j < dl; j++) enc[c][j] = (int)dec[j];
            free(codes);
            free(dec);
        }
        inverse_RLE(blocks[i].RLE_encoded_lum, blocks[i].lum_coefficients, 64, ll);
        inverse_RLE(blocks[i].RLE_encoded_r, blocks[i].r_coefficients, 32, lr);
        inverse_RLE(blocks[i].RLE_encoded_b, blocks[i].b_coefficients, 32, lb);
        double rl[64], rr[32], rb[32];
        reverse_zigzag_pattern(8, 8, blocks[i].lum_coefficients, rl);
        reverse_zigzag_pattern(4, 8, blocks[i].r_coefficients, rr);
        reverse_zigzag_pattern(4, 8, blocks[i].b_coefficients, rb);
        for (size_t j = 0; j < 64; j++) blocks[i].lum_coefficients[j] = rl[j];
        for (size_t j = 0; j < 32; j++) {
            blocks[i].r_coefficients[j] = rr[j];
            blocks[i].b_coefficients[j] = rb[j];
        }
    }
    for (size_t i = 0; i < total_blocks; i++) {                              /* :1408-1413 */
        Inverse_quantize(&(blocks[i].lum_coefficients), LUMINANCE_QUANTIZATION_TABLE, 64);
        Inverse_quantize(&(blocks[i].b_coefficients), CHROMINANCE_QUANTIZATION_TABLE, 32);
        Inverse_quantize(&(blocks[i].r_coefficients), CHROMINANCE_QUANTIZATION_TABLE, 32);
    }
    for (size_t i = 0; i < total_blocks; i++) {                              /* :1416-1421 */
        inverse_discrete_cosine_transform(blocks[i].lum_values, 8, 8, blocks[i].lum_coefficients);
        inverse_discrete_cosine_transform(blocks[i].b_values, 4, 8, blocks[i].b_coefficients);
        inverse_discrete_cosine_transform(blocks[i].r_values, 4, 8, blocks[i].r_coefficients);
    }
    ImageData rec = {0};
    assemble_image(&rec, img, blocks);                                       /* :1425 */
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            unsigned char *o = out_rgba + ((size_t)y * w + x) * 4;
            o[0] = rec.pixels[y][x].r;
            o[1] = rec.pixels[y][x].g;
            o[2] = rec.pixels[y][x].b;
            o[3] = rec.pixels[y][x].a;
        }
    for (size_t i = 0; i < total_blocks; i++) {
        free(blocks[i].lum_coefficients);
        free(blocks[i].r_coefficients);
        free(blocks[i].b_coefficients);
        free(blocks[i].RLE_encoded_lum);
        free(blocks[i].RLE_encoded_r);
        free(blocks[i].RLE_encoded_b);
    }
    free(blocks);
    for (int y = 0; y < h; y++) { free(lum[y]); free(cr[y]); free(cb[y]); }
    free(lum); free(cr); free(cb);
    free_pixels(img.pixels, h);
    free_pixels(rec.pixels, h);
    return 0;
}

/* The reference's entropy stage on one stream of n zigzagged ints, exactly as
 * its main loop runs it (JPEG.c:1211-1349): RLE, encode_huffman,
 * generate_encoded_sequence, decode_huffman written back over the RLE ints,
 * inverse_RLE.  Returns the RLE ints, the codes[] table (value, length, bits),
 * the '0'/'1' string packed MSB-first, and the n ints after the round trip.
 * The sequence buffer is larger than main()'s 1024 / 512 chars so that no
 * input overflows it here. */
int ref_jpeg_entropy(const short *zz, int n, int *rle, int *rle_len, int *ncodes,
                     short *tab_val, unsigned char *tab_len, unsigned long long *tab_code,
                     unsigned char *bits, int *nbits, short *decoded)
{
    double in[64], out[64];
    for (int i = 0; i < n; i++) in[i] = zz[i];
    int *enc = NULL;
    size_t enc_len = 0;
    RLE(in, (size_t)n, &enc, &enc_len);
    for (size_t i = 0; i < enc_len; i++) rle[i] = enc[i];
    *rle_len = (int)enc_len;
    size_t code_count = 0;
    Node *root = NULL;
    HuffmanCode *codes = encode_huffman(enc, enc_len, &code_count, &root);
    *ncodes = (int)code_count;
    for (size_t c = 0; c < code_count; c++) {
        tab_val[c] = (short)(codes[c].value - 1000);
        tab_len[c] = (unsigned char)strlen(codes[c].code);
        unsigned long long v = 0;
        for (const char *p = codes[c].code; *p; p++) v = (v << 1) | (unsigned long long)(*p == '1');
        tab_code[c] = v;
    }
    static char seq[16384];
    generate_encoded_sequence(enc, enc_len, codes, (int)code_count, seq);
    int nb = (int)strlen(seq);
    memset(bits, 0, (size_t)(nb + 7) / 8);
    for (int i = 0; i < nb; i++)
        if (seq[i] == '1') bits[i >> 3] |= (unsigned char)(0x80 >> (i & 7));
    *nbits = nb;
    size_t dlen = 0;
    double *dec = decode_huffman(root, seq, &dlen);
    for (size_t j = 0; j < dlen; j++) enc[j] = (int)dec[j];          /* :1237-1240 */
    inverse_RLE(enc, out, (size_t)n, enc_len);                        /* :1346 */
    for (int i = 0; i < n; i++) decoded[i] = (short)out[i];
    free(dec);
    free(codes);
    free(enc);
    return 0;
}

/* The reference's own visual PNGs (JPEG.c:1103-1123): original.png,
 * luminance.png, rChrominance.png, bChrominance.png, written by its
 * create_*_image functions through stb_image_write into
 * OUTPUT_DIRECTORY ("../Output-Input/Images/", relative to the cwd -- run
 * this from a scratch Experiment/ directory). */
int ref_jpeg_visual_pngs(const unsigned char *rgba, int w, int h)
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
    create_png_image("original.png", w, h, img.pixels);
    build_luminance_matrix(img, &lum);
    create_luminance_image("luminance.png", lum, img);
    build_rChrominance_matrix(img, &cr);
    create_rChrominance_image("rChrominance.png", cr, img);
    build_bChrominance_matrix(img, &cb);
    create_bChrominance_image("bChrominance.png", cb, img);
    for (int y = 0; y < h; y++) { free(lum[y]); free(cr[y]); free(cb[y]); }
    free(lum); free(cr); free(cb);
    free_pixels(img.pixels, h);
    return 0;
}

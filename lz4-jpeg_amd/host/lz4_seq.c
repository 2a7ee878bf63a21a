/*
 * LZ4_seq -- drop-in for the reference's LZ4_seq.exe
 * (Algorithms/sequential/LZ4/LZ4.c main, :1123-1136) on the MI355X path.
 *
 * Same file contract, run from Experiment/ as the drivers do
 * (Experiment/LZ4_sequential_experiment.c:102 popen("LZ4_seq.exe 2>&1")):
 *   truncates ../Output-Input/out/compressed.bin and the log (clear_files,
 *   LZ4.c:204-213), compresses ../Output-Input/input/input.txt into
 *   compressed.bin + its "%02X " dump compressed.txt (lz4_encode on the GPU),
 *   decodes it to uncompressed.txt (LZ4_decode, exact decoder), exit 0.
 * Input shorter than 300 B: the reference's message and exit(1).
 * Not replicated: ensure_directories (LZ4.c:181-202), whose mkdir of
 * ../../../Output-Input/input exits 1 whenever that directory is absent and
 * makes the drivers retry forever.
 */
#include <stdio.h>

#include "../../include/lz4jpeg_compat.h"

static void clear_files(void) {
  FILE *f = fopen(LZ4_COMPRESSED_FILE, "wb");
  if (f) fclose(f);
  f = fopen(LZ4_LOG_FILE, "w");
  if (f) fclose(f);
}

int main(void) {
  clear_files();
  lz4_encode();
  LZ4_decode(LZ4_COMPRESSED_FILE, LZ4_LOG_FILE);
  return 0;
}

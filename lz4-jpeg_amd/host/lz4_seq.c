/*
 * LZ4_seq / LZ4_par -- drop-ins for the reference's LZ4_seq.exe
 * (Algorithms/sequential/LZ4/LZ4.c main, :1123-1136) and LZ4_par.exe
 * (Algorithms/parallel/LZ4/LZ4.c main, :1227-1250; spawned by
 * Experiment/LZ4_parallel_experiment.c:102 popen("LZ4_par.exe 2>&1")) on the
 * MI355X path.  The parallel variant's per-block output is the sequential
 * one's (a thread per block, LZ4.c:518-628 of the parallel file), so both
 * executables run the same GPU compressor; LZ4_par (built with -DLZ4_PAR)
 * also prints the parallel main's closing "Number of cores available" line
 * (host logical processors, as GetSystemInfo reports them).
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
#include <unistd.h>

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
#ifdef LZ4_PAR
  printf("Number of cores available: %ld\n", sysconf(_SC_NPROCESSORS_ONLN));
#endif
  return 0;
}

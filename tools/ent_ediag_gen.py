"""Make a phase-stamp diag source of jpegr_entropy.hip (tools only):
    python3 tools/ent_ediag_gen.py in.hip out.hip
s_memtime stamps (lane 0 of each encode wave) into g_eph[kernel][wave][k]:
0 start, 1 before the RLE, 2 after it, 3 before tree_codes, 4 after it,
5 after the sequence bits, 6 after the meta word; read with jpegr_eph_read
(tools/ent_ephase.py)."""
import sys

src = open(sys.argv[1]).read()
i = src.index('namespace {')
src = src[:i] + '__device__ uint32_t g_eph[2][4096][8];\n' + src[i:]


def rep(a, b):
    global src
    assert src.count(a) == 1, (a, src.count(a))
    src = src.replace(a, b)


ST = ('{ const uint32_t _t = (uint32_t)__builtin_amdgcn_s_memtime(); '
      'if (lane == 0 && blockIdx.x < 4096) g_eph[kLuma ? 0 : 1][blockIdx.x][%d] = _t; }\n')
rep('  const int c = kLuma ? 0 : 1 + (int)(blockIdx.x & 1);      // channel of this wave',
    ST % 0 + '  const int c = kLuma ? 0 : 1 + (int)(blockIdx.x & 1);      // channel of this wave')
rep('  uint32_t lid[(N + 2) / 3];', ST % 1 + '  uint32_t lid[(N + 2) / 3];')
rep("  uint64_t dm = 0;                                    // (luma) the wave's deferred lanes",
    ST % 2 + "  uint64_t dm = 0;                                    // (luma) the wave's deferred lanes")
rep('    bool over = tree_codes<Cap>(w, U, table + tile * kTablePerTile + bits_off(c), h0);',
    ST % 3 + '    bool over = tree_codes<Cap>(w, U, table + tile * kTablePerTile + bits_off(c), h0);\n' + ST % 4)
rep('    const int nbits = pos;', ST % 5 + '    const int nbits = pos;')
rep('''    } else if (over) {
      atomicAdd(&status[0], 1u);
    }
  }''', '''    } else if (over) {
      atomicAdd(&status[0], 1u);
    }
''' + ST % 6 + '  }')
src += '''
extern "C" int jpegr_eph_read(void *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_eph), sizeof(g_eph)) == hipSuccess ? 0 : -1;
}
'''
open(sys.argv[2], 'w').write(src)

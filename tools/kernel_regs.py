"""Print VGPR/SGPR/spill/LDS metadata of kernels in a built object (llvm-readelf --notes dump).
   usage: python tools/kernel_regs.py NOTES.txt [substring ...]"""
import re
import sys

txt = open(sys.argv[1]).read()
subs = sys.argv[2:]
for blk in re.split(r'\n\s+- \.', txt):
    m = re.search(r'\.name:\s+(\S+)', blk)
    if not m or (subs and not any(s in m.group(1) for s in subs)):
        continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\d+)', blk) or [None, None])[1]
    print(m.group(1), 'vgpr', g('vgpr_count'), 'sgpr', g('sgpr_count'), 'vspill', g('vgpr_spill_count'),
          'lds', g('group_segment_fixed_size'))

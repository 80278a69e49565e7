import re, subprocess, sys, tempfile, os
def kernels(path):
    data = open(path, 'rb').read()
    res = {}
    for m in re.finditer(b'__CLANG_OFFLOAD_BUNDLE__', data):
        off = m.start()
        n = int.from_bytes(data[off+24:off+32], 'little')
        p = off + 32
        for _ in range(n):
            eoff = int.from_bytes(data[p:p+8], 'little'); esz = int.from_bytes(data[p+8:p+16], 'little')
            tl = int.from_bytes(data[p+16:p+24], 'little'); trip = data[p+24:p+24+tl].decode(); p += 24 + tl
            if 'gfx950' not in trip: continue
            blob = data[off+eoff: off+eoff+esz]
            with tempfile.NamedTemporaryFile(delete=False, dir='.') as f: f.write(blob); fn = f.name
            out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-readelf', '--notes', fn], capture_output=True, text=True).stdout
            os.unlink(fn)
            for k in re.finditer(r'\.name:\s+(\S+)\n(?:.*\n)*?', out): pass
            # parse kernels blocks
            for blk in out.split('  - .agpr_count')[1:]:
                name = re.search(r'\.name:\s+(\S+)', blk); vg = re.search(r'\.vgpr_count:\s+(\d+)', blk)
                sp = re.search(r'\.vgpr_spill_count:\s+(\d+)', blk); lds = re.search(r'\.group_segment_fixed_size:\s+(\d+)', blk)
                if name: res[name.group(1)] = (vg and int(vg.group(1)), sp and int(sp.group(1)), lds and int(lds.group(1)))
    return res
a = kernels(sys.argv[1]); b = kernels(sys.argv[2])
print(len(a), len(b))
for k in sorted(set(a) | set(b)):
    if a.get(k) != b.get(k): print(k[:90], a.get(k), b.get(k))

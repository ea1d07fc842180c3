"""Instruction mix of a kernel's outermost loops in a hipcc -S listing (what bounds a latency-bound
chain kernel: one compute wave per SIMD issues one VALU instruction per 4 cycles).  A loop is its
header block plus every basic block the listing annotates "in Loop: Header=<it>" (nested too).
usage: python tools/probes/loop_mix.py LISTING.s SYMBOL_SUBSTRING [top]"""
import collections
import re
import sys

src, key = sys.argv[1], sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
lines = open(src).read().split('\n')
start = next(k for k, l in enumerate(lines)
             if key in l and l.split(';')[0].strip().endswith(':') and not l.startswith('\t'))
end = next(k for k in range(start, len(lines)) if 's_endpgm' in lines[k])
body = lines[start:end + 1]
# basic blocks: (label line index, header it belongs to or None, own header name)
blocks, cur = [], None
for k, l in enumerate(body):
    if re.match(r'^(\.LBB\d+_\d+|; %bb\.\d+):', l.strip()) or (l.startswith('.LBB') and ':' in l):
        m = re.search(r'Header=(BB\d+_\d+)', l) or re.search(r'Parent Loop (BB\d+_\d+)', l)
        own = re.match(r'^\.L(BB\d+_\d+):', l.strip())
        depth1 = 'Loop Header: Depth=1' in l
        cur = {'hdr': m.group(1) if m else None, 'own': own.group(1) if own else None, 'd1': depth1, 'ins': []}
        blocks.append(cur)
        continue
    x = l.strip()
    if cur is not None and x and not x.startswith(';') and not x.startswith('.'):
        cur['ins'].append(x.split()[0])
heads = [b['own'] for b in blocks if b['d1']]
for h in heads:
    c = collections.Counter()
    # nested loops' blocks name their own header; include blocks whose header chain leads to h
    parent = {b['own']: b['hdr'] for b in blocks if b['own']}
    def under(hdr):
        seen = set()
        while hdr and hdr not in seen:
            if hdr == h:
                return True
            seen.add(hdr)
            hdr = parent.get(hdr)
        return False
    for b in blocks:
        if b['own'] == h or under(b['hdr']):
            c.update(b['ins'])
    print(f"loop {h}: {sum(c.values())} instructions")
    print('  ', sorted(c.items(), key=lambda t: -t[1])[:top])

if len(sys.argv) > 4 and sys.argv[4] == "nested":
    # every loop (any depth): instructions of the blocks whose innermost header it is
    own = collections.defaultdict(collections.Counter)
    for b in blocks:
        h = b['own'] if any(x.get('hdr') == b['own'] for x in blocks) and b['own'] else b['hdr']
        own[h].update(b['ins'])
    for h, c in own.items():
        if h:
            print(f"  loop {h} (own blocks): {sum(c.values())} instructions; "
                  f"VALU {sum(v for k, v in c.items() if k.startswith('v_'))}, MFMA {c['v_mfma_f32_16x16x32_bf16']}, "
                  f"LDS {sum(v for k, v in c.items() if k.startswith('ds_'))}, VMEM {sum(v for k, v in c.items() if k.startswith(('global_', 'buffer_')))}")

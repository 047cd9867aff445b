"""Map of one kernel's ISA: line numbers of labels, branches, spills (scratch), vmcnt waits and the
MFMA-dense region.   usage: python tools/isa_map.py <file.s> <kernel-name-substring>"""
import sys

s = open(sys.argv[1]).read().split('\n')
start = next(k for k, l in enumerate(s) if l.endswith(sys.argv[2] + ':') or (l.startswith('_Z') and sys.argv[2] in l and l.rstrip().endswith(':') ) or (l.startswith('_Z') and sys.argv[2] in l.split(':')[0] and ':' in l))
end = next(k for k in range(start, len(s)) if s[k].startswith('.Lfunc_end'))
body = s[start:end]
nm = [k for k, l in enumerate(body) if 'v_mfma' in l]
print(body[0][:80], 'lines', len(body), 'mfma', len(nm))
for k, l in enumerate(body):
    t = l.strip()
    if t.startswith(('scratch_', '.LBB', 's_cbranch', 's_branch', 's_barrier')) or ('vmcnt' in t and 's_waitcnt' in t) \
            or t.startswith('global_store') or t.startswith('global_load_lds') or t.startswith('global_load_dword'):
        print(k, t[:60])

#!/usr/bin/env python3
"""Loops of one kernel in a hipcc -S listing, found as strongly connected
components of its basic-block graph (a sub-step loop whose body branches --
StepNoise's group blocks, the wave-uniform fast/slow conversions -- is laid
out as several blocks, which a back-edge scan splits).  For every loop that
issues ds_bpermute_b32 (the run kernels' sub-step loops) prints its blocks
with their VALU / SALU / LDS / wait counts, the v_mad_u64_u32 count (Philox)
and the successors, so a sub-step's instruction budget can be read off per
path ("Where the E = 64 run's time goes").

usage: isa_loops.py ASM KERNEL_SYMBOL
  ASM: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off
       -fno-slp-vectorize -gline-tables-only --cuda-device-only -S -o ASM
       swarmrl_amd/csrc/swarm_engine.hip
  KERNEL_SYMBOL: the mangled name, e.g.
       _ZN5swarm13k_cluster_runILb0ELb0ELb0EEEvPKNS_7DerivedENS_8DevStateENS_7ScratchEiiPKmPKfiPy
"""
import re, sys, collections
asm, kern = sys.argv[1], sys.argv[2]
lines = open(asm).read().split('\n')
start = next(i for i, l in enumerate(lines) if l.startswith(kern + ':'))
end = start
while not lines[end].strip().startswith('.Lfunc_end'): end += 1
body = lines[start+1:end]
# file table for .loc
files = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
    if m: files[int(m.group(1))] = (m.group(3) or m.group(2))
blocks = []  # (label, [instrs], [(ins, loc)])
cur = ['entry', []]
loc = None
for l in body:
    m = re.match(r'^(\.LBB\d+_\d+):', l)
    if m:
        blocks.append(cur); cur = [m.group(1), []]; continue
    m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
    if m: loc = (int(m.group(1)), int(m.group(2))); continue
    if l.startswith('\t') and not l.startswith('\t.') and not l.startswith('\t;') and l.strip():
        cur[1].append((l.strip(), loc))
blocks.append(cur)
idx = {b[0]: k for k, b in enumerate(blocks)}
succ = collections.defaultdict(list)
for k, (lab, ins) in enumerate(blocks):
    term = False
    for s, _ in ins:
        op = s.split()[0]
        m = re.match(r's_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', s)
        if m:
            succ[k].append(idx[m.group(2)])
            if m.group(1) == 'branch': term = True
        if op == 's_endpgm': term = True
    if not term and k + 1 < len(blocks): succ[k].append(k + 1)
# Tarjan
sys.setrecursionlimit(100000)
index = {}; low = {}; st = []; on = set(); sccs = []; c = [0]
def strong(v):
    index[v] = low[v] = c[0]; c[0] += 1; st.append(v); on.add(v)
    for w in succ[v]:
        if w not in index: strong(w); low[v] = min(low[v], low[w])
        elif w in on: low[v] = min(low[v], index[w])
    if low[v] == index[v]:
        comp = []
        while True:
            w = st.pop(); on.discard(w); comp.append(w)
            if w == v: break
        sccs.append(comp)
for v in range(len(blocks)):
    if v not in index: strong(v)
def kind(s):
    op = s.split()[0]
    if op.startswith('v_'): return 'valu'
    if op.startswith('s_waitcnt') or op.startswith('s_nop'): return 'wait'
    if op.startswith('s_'): return 'salu'
    if op.startswith('ds_'): return 'lds'
    return 'vmem'
for comp in sccs:
    if len(comp) < 2 and blocks[comp[0]][0] not in [blocks[w][0] for w in succ[comp[0]]]: continue
    ops = collections.Counter()
    for b in comp:
        for s, _ in blocks[b][1]: ops[s.split()[0]] += 1
    if ops['ds_bpermute_b32'] == 0: continue
    tot = collections.Counter()
    for b in comp:
        for s, _ in blocks[b][1]: tot[kind(s)] += 1
    print('SCC', len(comp), 'blocks', dict(tot), 'bperm', ops['ds_bpermute_b32'], 'ds_add', ops['ds_add_u64'], 'mad64', ops['v_mad_u64_u32'])
    for b in sorted(comp):
        t = collections.Counter(kind(s) for s, _ in blocks[b][1])
        mad = sum(1 for s, _ in blocks[b][1] if s.startswith('v_mad_u64'))
        print('   ', blocks[b][0], dict(t), 'mad64', mad, '->', [blocks[w][0] for w in succ[b]])

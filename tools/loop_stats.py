#!/usr/bin/env python3
"""Instruction mix of every loop body of one kernel in an llvm-objdump disassembly (developer tool):
loops are found from backward branches; per loop: packed FMAs, MFMAs, SGPR-spill reloads
(v_readlane) and stores (v_writelane), LDS / scalar / buffer loads, other VALU, barriers, waits.

usage: python3 tools/loop_stats.py <disassembly.s> <kernel-name-substring>
(disassembly: llvm-objcopy --only-section=.hip_fatbin, clang-offload-bundler --unbundle
--targets=hipv4-amdgcn-amd-amdhsa--gfx950, llvm-objdump -d; as in tests/test_kernel_resources_cpu.py)"""
import re
import sys
L=open(sys.argv[1]).read().split('\n')
st=[i for i,l in enumerate(L) if re.match(r'^[0-9a-f]+ <.*%s.*>:'%sys.argv[2],l)][0]
en=next((i for i in range(st+1,len(L)) if re.match(r'^[0-9a-f]+ <',L[i])),len(L))
F=[]
for l in L[st+1:en]:
    m=re.match(r'\s*(\S.*?)\s*//\s*([0-9A-F]+):',l)
    if m: F.append((int(m.group(2),16),m.group(1)))
addr={a:i for i,(a,_) in enumerate(F)}
loops=[]
for i,(a,ins) in enumerate(F):
    m=re.match(r's_cbranch_\w+ (\d+)|s_branch (\d+)',ins)
    if m:
        off=int(m.group(1) or m.group(2))
        if off>=32768: off-=65536
        tgt=a+4+off*4
        if tgt<a and tgt in addr: loops.append((addr[tgt],i))
for s,e in sorted(set(loops)):
    body=[ins for _,ins in F[s:e+1]]
    c=lambda p: sum(1 for x in body if x.startswith(p))
    print(f"loop {s}-{e}: n={len(body)} pk_fma={c('v_pk_fma')} mfma={c('v_mfma')} readlane={c('v_readlane')} writelane={c('v_writelane')} ds_read={c('ds_read')} s_load={c('s_load')} buf_load={c('buffer_load')} valu_other={sum(1 for x in body if x.startswith('v_') and not x.startswith(('v_pk_fma','v_mfma','v_readlane','v_writelane')))} barrier={c('s_barrier')} waitcnt={c('s_waitcnt')}")

"""Diagnostic: device-memory lines per op by pool, from the CPU emulator's statistics build
(tests/emu: make stats).  Every WaveCPU method reports the bytes its WaveGPU twin reads / writes; one
fast_txn / apply_txn call is an epoch, and each 128 B line it touches counts once as read and / or
written.  A model of L2-miss traffic with no reuse across ops (writes of tails appended op after op
coalesce in L2 on the GPU, so the write column over-counts those).

usage: python scripts/emu_mem_lines.py c5 [rounds] | c4 | ap"""
import ctypes as C, os, sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT + '/text-crdt-rust_amd'); sys.path.insert(0, ROOT + '/tests')
L=C.CDLL(ROOT + '/tests/emu/build/libemu_stats.so')
L.emu_new.restype=C.c_void_p; L.emu_new.argtypes=[C.c_uint32]
L.emu_run_wire.argtypes=[C.c_void_p,C.c_char_p,C.c_size_t,C.c_uint32]
L.emu_run_random.argtypes=[C.c_void_p,C.c_uint16,C.c_uint32,C.c_uint32,C.c_uint32]
L.emu_agent.argtypes=[C.c_void_p,C.c_char_p]
P=C.POINTER(C.c_ulonglong)
L.emu_mem_stats.restype=C.c_ulonglong; L.emu_mem_stats.argtypes=[P,P,C.c_int]
names="leaves dir sol leaf_of agent_of lag cwo arun dels dd ddb txns parents frontier agents groups recs other".split()
rd=np.zeros(18,np.uint64); wr=np.zeros(18,np.uint64)
L.emu_mem_stats(rd.ctypes.data_as(P),wr.ctypes.data_as(P),1)
what=sys.argv[1]
h=L.emu_new(32)
if what=='c5':
    from fuzz_gen import config5_wire
    rounds=int(sys.argv[2]) if len(sys.argv)>2 else 64
    w=config5_wire(900, base_len=1<<20, n_agents=16, rounds=rounds, ops=64)
    print('status',L.emu_run_wire(h,w,len(w),48)); nops=16*rounds*64+1
elif what=='c4':
    ag=L.emu_agent(h,b"gen"); print('status',L.emu_run_random(h,ag,20000,1,32)); nops=20000
else:
    from crdt_amd.traces import load_remote_wire
    w=load_remote_wire('automerge-paper'); print('status',L.emu_run_wire(h,w,len(w),32)); nops=259778
ep=L.emu_mem_stats(rd.ctypes.data_as(P),wr.ctypes.data_as(P),1)
print('epochs',ep,'ops',nops)
tr=tw=0
for i,n in enumerate(names):
    if rd[i] or wr[i]:
        print(f'{n:10s} read {rd[i]*128/nops:9.1f} B/op  write {wr[i]*128/nops:9.1f} B/op')
    tr+=rd[i]; tw+=wr[i]
print(f'TOTAL      read {tr*128/nops:9.1f} B/op  write {tw*128/nops:9.1f} B/op')

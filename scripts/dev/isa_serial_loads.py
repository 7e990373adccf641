#!/usr/bin/env python3
"""Per kernel of the library's device code: global/buffer loads, and how many of them are followed
within two instructions by `s_waitcnt vmcnt(0)` -- the signature of a guarded load compiled to an
exec-masked branch that waits for its own result, which serialises a group of loads meant to be in
flight together (found in k_kmeans' tile loops, round 5).  usage: isa_serial_loads.py [file.hip ...]"""
import os, re, subprocess, sys

CSRC = os.path.join(os.path.dirname(__file__), '..', '..', 'vent_analysis_amd', 'csrc')
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-ffp-contract=off', '-I/opt/rocm/include',
         '--cuda-device-only', '--no-gpu-bundle-output', '-S']


def scan(src):
    out = '/tmp/isa_' + os.path.basename(src) + '.s'
    subprocess.run(['/opt/rocm/bin/hipcc', *FLAGS, '-o', out, src], check=True, stderr=subprocess.DEVNULL)
    s = open(out).read()
    for m in re.finditer(r'^(_Z\w+):.*\n', s, re.M):
        end = s.find('.Lfunc_end', m.end())
        body = s[m.end():end].splitlines()
        loads = [n for n, l in enumerate(body) if re.search(r'\b(global|buffer|flat)_load', l)]
        ser = sum(1 for n in loads if any('vmcnt(0)' in body[q] for q in range(n + 1, min(n + 3, len(body)))))
        if loads:
            yield m.group(1), len(loads), ser


if __name__ == '__main__':
    files = sys.argv[1:] or sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith('.hip'))
    for f in files:
        for name, n, ser in scan(f):
            if ser:
                print(f'{os.path.basename(f):14s} {name[:60]:60s} loads {n:4d}  followed by vmcnt(0) {ser:4d}')

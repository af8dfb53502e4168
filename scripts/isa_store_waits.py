"""Count, per kernel of a gfx950 assembly listing, the `s_waitcnt vmcnt(0)` that follow a global
store with no load in between.  gfx950 counts loads and stores in one vmcnt, so such a wait
(typically inside a per-record branch that uses a value loaded earlier) also waits for the
store's round trip -- how k_dl_words' per-record waits were found.
usage: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude --cuda-device-only -S -o x.s
       genome-compression_amd/csrc/gcz_build.hip && python3 scripts/isa_store_waits.py x.s"""
import re
import sys


def main(path):
    s = open(path).read()
    for m in re.finditer(r"\n(_Z\S+):[^\n]*\n(.*?)s_endpgm", s, re.S):
        pending, waits, stores = False, 0, 0
        for line in m.group(2).splitlines():
            t = line.strip()
            if t.startswith(("global_store", "buffer_store")):
                pending, stores = True, stores + 1
            elif t.startswith(("global_load", "buffer_load", "global_atomic", "flat_load")):
                pending = False
            elif t.startswith("s_waitcnt") and "vmcnt(0)" in t and pending:
                waits, pending = waits + 1, False
        if waits:
            print(f"{waits:4d} waits after a store / {stores:4d} stores  {m.group(1)[:80]}")


if __name__ == "__main__":
    main(sys.argv[1])

#!/usr/bin/env python3
"""Generate tests/golden/dispatch.json from the REFERENCE ITSELF (run in the build container only).

The reference decides which compiled function serves each (collective, redop, datatype, algorithm,
protocol) by running its own generator, src/device/generate.py (required_cuda :100-125,
equivalent_primary :128-136, the tables it writes at :201-305). This script runs that generator,
unmodified, as its Makefile does (`python3 generate.py <outdir>`, src/device/Makefile), into a
scratch directory, and reads the three tables it writes:

  host_table.cc    ncclDevFuncRowToId[]: row (coll, redop, ty, algo, proto) -> function id (-1: none)
  device_table.cc  ncclDevFuncTable[]:   function id -> ncclDevFunc_<name>, with its #if guard
  <coll>_<redop>_<ty>.cc  DEFINE_ncclDevFunc(<name>, coll, Func<Op>, <C++ type>, algo, proto)

and writes, for the reductions (AllReduce / Reduce / ReduceScatter) on the RING and TREE algorithms
(the schedules whose SIMPLE / LL / LL128 primitives reach reduceCopy and the LL reduce), the functor
and C++ element type the reference instantiates, and the compile guard on it. Nothing of the
reference's text is kept: the fixture is the generator's decisions, as data.

    python3 tests/golden/make_dispatch_golden.py [/root/reference]

The GPU box has no /root/reference; only this container runs the script. tests/test_dispatch.py
checks the build's dispatch, validation and integer arithmetic against the fixture.
"""
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "dispatch.json")
COLLS = ("AllReduce", "Reduce", "ReduceScatter")
ALGOS = ("RING", "TREE")


def run_generator(ref: str, outdir: str) -> None:
    gen = os.path.join(ref, "src", "device", "generate.py")
    subprocess.run([sys.executable, gen, outdir], check=True, cwd=os.path.dirname(outdir), timeout=120,
                   stdout=subprocess.DEVNULL)


def parse(outdir: str) -> dict:
    # row -> id, with the row's name in the trailing comment
    rows = []
    text = open(os.path.join(outdir, "host_table.cc")).read()
    body = text.split("ncclDevFuncRowToId[] = {", 1)[1].split("};", 1)[0]
    for line in body.splitlines():
        m = re.match(r"/\*\s*(\d+)\*/\s*(-?\d+),\s*(?://\s*(.*))?$", line.strip())
        if m:
            rows.append((int(m.group(1)), int(m.group(2)), (m.group(3) or "").split()))
    # id -> (function name, guard)
    ids = {}
    text = open(os.path.join(outdir, "device_table.cc")).read()
    body = text.split("ncclDevFuncTable[] = {", 1)[1].split("};", 1)[0]
    guard = None
    for line in body.splitlines():
        line = line.strip()
        if line.startswith("#if "):
            guard = line[4:]
        elif line.startswith("#else"):
            guard = "else:" + (guard or "")
        elif line.startswith("#endif"):
            guard = None
        else:
            m = re.match(r"/\*\s*(\d+)\*/\s*(ncclDevFunc_\w+|nullptr),", line)
            if m and m.group(2) != "nullptr" and not (guard or "").startswith("else:"):
                ids[int(m.group(1))] = (m.group(2)[len("ncclDevFunc_"):], guard)
    # function name -> (functor, C++ type)
    defs = {}
    for fn in os.listdir(outdir):
        if not fn.endswith(".cc"):
            continue
        for m in re.finditer(r"DEFINE_ncclDevFunc\((\w+),\s*\w+,\s*(\w+),\s*(\w+),", open(os.path.join(outdir, fn)).read()):
            defs[m.group(1)] = (m.group(2), m.group(3))
    out = []
    for row, fid, name in rows:
        if len(name) != 5 or name[0] not in COLLS or name[3] not in ALGOS:
            continue
        coll, redop, ty, algo, proto = name
        ent = {"coll": coll, "redop": redop, "ty": ty, "algo": algo, "proto": proto, "row": row, "id": fid}
        if fid >= 0:
            fname, g = ids[fid]
            functor, ctype = defs[fname]
            ent.update(function=fname, functor=functor, ctype=ctype, guard=g)
        out.append(ent)
    return {"rows": out}


def main() -> int:
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    gen_src = open(os.path.join(ref, "src", "device", "generate.py")).read()
    lists = {}
    for key in ("all_redops", "all_tys", "all_protos", "all_algos"):
        m = re.search(rf"^{key}\s*=\s*(\[[^\]]*\])", gen_src, re.M)
        lists[key] = json.loads(m.group(1).replace("'", '"'))
    with tempfile.TemporaryDirectory() as d:
        outdir = os.path.join(d, "gensrc")
        run_generator(ref, outdir)
        data = parse(outdir)
    data = {"source": "reference src/device/generate.py run unmodified (tests/golden/make_dispatch_golden.py)",
            "order": lists, **data}
    with open(OUT, "w") as f:
        json.dump(data, f, indent=0, sort_keys=True)
        f.write("\n")
    print(f"wrote {OUT}: {len(data['rows'])} rows")
    return 0


if __name__ == "__main__":
    sys.exit(main())

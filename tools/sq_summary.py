#!/usr/bin/env python3
"""Per-kernel SQ summary from tools/pmc_table.py's CSV (counters averaged per launch).
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles (MI355X_MICROARCH.md); FETCH_SIZE
and WRITE_SIZE are KB; HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (the guide's gfx950
correction)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
print("| kernel | waves | wave-cycles/wave | wait_inst | wait_any | active | VALU/wave | LDS/wave "
      "| bank-conflict cyc/LDS instr | LDS cyc/LDS instr | HBM MB/launch |")
print("|---|---|---|---|---|---|---|---|---|---|---|")
for r in rows:
    def f(k):
        return float(r[k]) if r.get(k) else float("nan")
    wc, wv = f("SQ_WAVE_CYCLES"), f("SQ_WAVES")
    print("| %s | %.0f | %.0f | %.2f | %.2f | %.2f | %.0f | %.0f | %.2f | %.2f | %.1f |" % (
        r["kernel"], wv, 4 * wc / wv, f("SQ_WAIT_INST_ANY") / wc, f("SQ_WAIT_ANY") / wc,
        f("SQ_ACTIVE_INST_ANY") / wc, f("SQ_INSTS_VALU") / wv, f("SQ_INSTS_LDS") / wv,
        f("SQ_LDS_BANK_CONFLICT") / max(f("SQ_INSTS_LDS"), 1), f("SQ_LDS_IDX_ACTIVE") / max(f("SQ_INSTS_LDS"), 1),
        (2 * f("FETCH_SIZE") + f("WRITE_SIZE")) / 1e3))

"""Per-kernel time summary from a rocprofv3 rocpd database: python tools/kstats_db.py <dir> [steps]"""
import glob
import sqlite3
import sys

db = glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True)[0]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), sum(end-start)/1e6, max(vgpr_count), max(accum_vgpr_count), "
                 "max(scratch_size), max(lds_size) from kernels group by name order by 3 desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total {tot / steps:.2f} ms per step ({steps} steps)")
for n, cnt, ms, v, av, sc, lds in rows[:25]:
    print(f"{ms / steps:8.2f} ms {cnt // steps:5d}/step vgpr {v:3d} agpr {av:3d} scratch {sc:5d} lds {lds:6d}  {n[:70]}")

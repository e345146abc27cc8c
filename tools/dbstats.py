#!/usr/bin/env python3
"""Per-kernel call count / total / average (us) from rocprofv3 sqlite output (run_results.db)."""
import sqlite3
import sys

for path in sys.argv[1:]:
    c = sqlite3.connect(path)
    print(path)
    for name, calls, total_us, avg_us, pct in c.execute("select * from top_kernels limit 8"):
        print(f"  {calls:>5} {float(total_us):>10.1f} us  avg {float(avg_us):>9.2f} us  {name[:90]}")

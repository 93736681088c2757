"""CPU restatement of the reference loop as a 'fleet': 1 thread and N threads
(one per core, disjoint equal chunks) -- SURVEY §8(d) CPU lines.  Dev tool."""
import json, os, sys, time, platform
sys.path.insert(0, '.')
from oracle import oracle
oracle.build()
threads = int(sys.argv[1]) if len(sys.argv) > 1 else 16
cpu = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")), "?")
out = {"host_cpu": cpu, "nproc": os.cpu_count()}
for name, msg, n1, nN in [("cfg2 bradfitz", b"bradfitz", 20_000_000, 200_000_000)]:
    t = time.perf_counter(); oracle.c_scan(msg, 0, n1 - 1, threads=1); d1 = time.perf_counter() - t
    t = time.perf_counter(); oracle.c_scan(msg, 0, nN - 1, threads=threads); dN = time.perf_counter() - t
    out[name] = {"1_thread_MHs": n1 / d1 / 1e6, f"{threads}_threads_MHs": nN / dN / 1e6}
print(json.dumps(out))

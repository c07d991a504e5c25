"""Timeline of the last duplex call in a rocprofv3 kernel + memory-copy
trace (`rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d
DIR -o run -- python3 tools/host_rate.py ...`): kernels (with their HW
queue) and H2D copies, ms from the call's first copy-out.

usage: python tools/duplex_timeline.py DIR
"""
import csv, sys
d=sys.argv[1]
rows=list(csv.DictReader(open(d+'/run_kernel_trace.csv')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
sd=[r for r in rows if 'slab' in r['Kernel_Name']]
t0=int(sd[-16]['Start_Timestamp'])
ev=[]
for r in rows:
    s=int(r['Start_Timestamp']); e=int(r['End_Timestamp'])
    if s>=t0-800_000 and s<=int(sd[-1]['End_Timestamp']):
        ev.append((s,e,r['Kernel_Name'][:22]+" q"+r['Queue_Id']))
for r in csv.DictReader(open(d+'/run_memory_copy_trace.csv')):
    s=int(r['Start_Timestamp']); e=int(r['End_Timestamp'])
    if s>=t0-800_000 and s<=int(sd[-1]['End_Timestamp']):
        ev.append((s,e,"H2D"))
ev.sort()
for s,e,n in ev[:40]:
    print("%-28s %8.3f %8.3f dur %.3f" % (n,(s-t0)/1e6,(e-t0)/1e6,(e-s)/1e6))

import csv,sys
tag=sys.argv[1]
K=list(csv.DictReader(open(f'gpurun_out/trace/{tag}_kernel_trace.csv')))
M=list(csv.DictReader(open(f'gpurun_out/trace/{tag}_memory_copy_trace.csv')))
ev=[(int(r['Start_Timestamp']),int(r['End_Timestamp']),r['Kernel_Name'].split('(')[0].replace('cordahip::','').replace('void ','')[-28:],'K', r.get('Stream_Id')) for r in K]
ev+=[(int(r['Start_Timestamp']),int(r['End_Timestamp']),r.get('Direction','copy')[12:],'M', r.get('Stream_Id')) for r in M]
ev.sort()
preps=[e for e in ev if 'ed25519_prep' in e[2]]
last = preps[-4:]
s0=last[0][0]-20_000_000
for e in ev:
    if e[0]>=s0 and (e[1]-e[0]>150000):
        print('  %8.2f %8.2f %6.2f %s %-30s %s'%((e[0]-s0)/1e6,(e[1]-s0)/1e6,(e[1]-e[0])/1e6,e[3],e[2],e[4]))

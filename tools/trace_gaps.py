import csv, sys
rows=list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rows) if 'k_minmax' in r['Kernel_Name']]
for k in range(3, min(len(idx)-1, 8)):
    seg=rows[idx[k]:idx[k+1]]
    t0=int(seg[0]['Start_Timestamp']); prev=None; gaps=[]; first=None; last=None
    for r in seg:
        s,e=int(r['Start_Timestamp']),int(r['End_Timestamp'])
        if 'pass_direct' in r['Kernel_Name']:
            if first is None: first=(s-t0)/1000
            last=(e-t0)/1000
            if prev and (s-prev)/1000>2: gaps.append(round((s-prev)/1000,1))
        prev=e
    print('step', k, 'passes', round(first,1), '->', round(last,1), 'gaps', gaps, 'span', round((int(rows[idx[k+1]]['Start_Timestamp'])-t0)/1000,1))

import csv, re, sys
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
agg = defaultdict(list)
order = []
for r in rows:
    nm = r['Kernel_Name']
    m = re.search(r'k_gemm<([^>]*)>', nm)
    key = ('ours ' + m.group(1)) if m else ('torch ' + nm[:30])
    key += f" grid={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
    if key not in agg:
        order.append(key)
    agg[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k in order:
    v = agg[k]
    if len(v) >= 20:
        print(f'{sorted(v)[len(v) // 2]:8.1f} us  {k}')

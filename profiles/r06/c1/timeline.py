import csv,sys
rows=[]
for r in csv.DictReader(open(sys.argv[1])):
    n=r["Kernel_Name"].split("(")[0].replace("void ","").replace("hfg::","")
    rows.append((int(r["Start_Timestamp"]),int(r["End_Timestamp"]),n,r["Queue_Id"],int(r["Grid_Size_X"])*int(r["Grid_Size_Y"])*int(r["Grid_Size_Z"])//int(r["Workgroup_Size_X"])))
rows.sort()
idx=[i for i,r in enumerate(rows) if r[2]=='absmax_kernel']
s=idx[-2]; e=idx[-1]
t0=rows[s][0]
for r in rows[s:e]:
    print(f"{(r[0]-t0)/1e3:8.1f} {(r[1]-t0)/1e3:8.1f} {(r[1]-r[0])/1e3:7.1f} q{r[3]} blk{r[4]:6d} {r[2][:60]}")

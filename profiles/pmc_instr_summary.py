import csv, glob, collections, sys
for d in sys.argv[1:]:
    acc=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.defaultdict(set)
    for f in glob.glob(d+'/**/run_counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k='analyze' if 'analyze' in r['Kernel_Name'] else 'resolve' if 'resolve' in r['Kernel_Name'] else None
            if not k: continue
            acc[k][r['Counter_Name']]+=float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
    for k,dd in acc.items():
        w=dd['SQ_WAVES']
        print(d, k, 'waves %.0f'%w, ' '.join('%s=%.0f'%(c.replace('SQ_INSTS_',''), dd[c]/w) for c in ['SQ_INSTS_VALU','SQ_INSTS_SALU','SQ_INSTS_LDS','SQ_WAVE_CYCLES']), 'gui_ms=%.2f'%(dd['GRBM_GUI_ACTIVE']/len(n[k])/8/2.4e6))

# Diagnostic: warm-start iterations / fix-ups over the bench's random walk for several settings.
summ() { python -c "
import sys,re
n=0;fx=0;mi=[];mx=0
for l in sys.stdin:
    m=re.search(r'mean_it ([0-9.]+) max_it (\d+) bad \[(.*?)\] fixed_up \[(.*?)\]',l)
    if not m: continue
    n+=1; mi.append(float(m.group(1))); mx=max(mx,int(m.group(2))); fx+=len([x for x in m.group(4).split(',') if x.strip()])
print('$1', 'ticks',n,'mean_it',round(sum(mi)/max(n,1),3),'max',mx,'fixups',fx)"; }
# usage: bash tools/warm_sweep.sh "<restart iterations>"   (OSC_WARM_* overrides: diagnostic only)
for r in ${1:-22}; do
  OSC_WARM_RESTART=$r timeout -k 10 150 python tools/warm_stalls.py walter_sr 32768 1 2>&1 | summ "walter restart=$r"
  OSC_WARM_RESTART=$r timeout -k 10 150 python tools/warm_stalls.py unitree_go2 65536 1 2>&1 | summ "go2 restart=$r"
done

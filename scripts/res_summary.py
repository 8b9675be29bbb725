import re,sys
t=open(sys.argv[1]).read()
pat=sys.argv[2] if len(sys.argv)>2 else ''
cur=None; info={}
for line in t.splitlines():
    m=re.search(r"Function Name: (\S+)",line)
    if m: cur=m.group(1); info[cur]={}; continue
    for key,k in (("VGPRs:","v"),("AGPRs:","a"),("ScratchSize","scr"),("Occupancy","occ"),("SGPRs:","s")):
        if key in line and cur:
            info[cur][k]=line.split(':')[-1].split('[')[0].strip() if key!="ScratchSize" else line.split(']:')[-1].split('[')[0].strip()
for n,d in info.items():
    if pat in n: print(f"{n[-60:]:60s} v={d.get('v')} a={d.get('a')} scr={d.get('scr')} occ={d.get('occ')}")

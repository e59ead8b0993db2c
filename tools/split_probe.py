#!/usr/bin/env python3
# For the long C3 path's extension rays (inside the red Suzanne): node visits of the
# reference closest-hit walk of the Suzanne BLAS split into the near- and the far-root-child
# subtree, and the visits of an unculled far-subtree walk (what a partner wave would do).
import sys, numpy as np
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/surf-path-tracer_amd')
import oracle
o = oracle.OracleScene()
ex = o.export()
nodes = np.frombuffer(ex['blas_nodes'], np.float32).reshape(-1,12); nu = nodes.view(np.uint32)
inst = np.frombuffer(ex['instances'], np.float32).reshape(-1,40); iu = inst.view(np.uint32)
idx = np.frombuffer(ex['blas_indices'], np.uint32)
tris = np.frombuffer(ex['triangles'], np.float32).reshape(-1,16)
k=3  # susanne0
triOff, idxOff, nodeOff = iu[k,0], iu[k,1], iu[k,2]
Minv = inst[k,24:40].reshape(4,4)  # column major: Minv[col][row]
z=np.load('/root/repo/tools/chainpath_rays.npz')
def xf(p,w):
    v=np.array([p[0],p[1],p[2],w],np.float32)
    r=np.array([sum(np.float32(Minv[c][rr])*v[c] for c in range(4)) for rr in range(4)],np.float32)
    return r[:3]
def slab(mn,mx,o,rd,depth):
    t0=(mn-o)*rd; t1=(mx-o)*rd
    tmin=max(min(t0[0],t1[0]),min(t0[1],t1[1]),min(t0[2],t1[2])); tmax=min(max(t0[0],t1[0]),max(t0[1],t1[1]),max(t0[2],t1[2]))
    return tmin if (tmax>=tmin and tmin<depth and tmax>0) else 1e30
def tri_hit(t_i,o,d,depth):
    T=tris[triOff+idx[idxOff+t_i]]
    v0,v1,v2=T[0:3],T[4:7],T[8:11]
    e1=v1-v0; e2=v2-v0; h=np.cross(d,e2); a=np.dot(e1,h)
    if abs(a)<1e-5: return None
    f=1/a; s=o-v0; u=f*np.dot(s,h)
    if u<0 or u>1: return None
    q=np.cross(s,e1); v=f*np.dot(d,q)
    if v<0 or u+v>1: return None
    t=f*np.dot(e2,q)
    return t if (1e-5<=t<depth) else None
def walk(start,o,d,rd,depth):
    st=[start]; visits=0
    while st:
        n=st.pop(); g=nodeOff+n
        if nu[g,1]:
            for j in range(nu[g,1]):
                t=tri_hit(nu[g,0]+j,o,d,depth)
                if t is not None: depth=t
            continue
        visits+=1
        l=nodeOff+nu[g,0]; r=l+1
        dl=slab(nodes[l,4:7],nodes[l,8:11],o,rd,depth); dr=slab(nodes[r,4:7],nodes[r,8:11],o,rd,depth)
        a,b=(nu[g,0],nu[g,0]+1)
        if dl>dr: dl,dr=dr,dl; a,b=b,a
        if dl==1e30: continue
        if dr!=1e30: st.append(b)
        st.append(a)
    return visits,depth
root=nodeOff; L=nu[root,0]; R=L+1
res=[]
for i in range(0,3086,7):
    o_=xf(z['eo'][i],1.0); d_=xf(z['ed'][i],0.0); rd=np.float32(1)/d_
    full,dfull=walk(0,o_,d_,rd,np.float32(1e30))
    dl=slab(nodes[nodeOff+L,4:7],nodes[nodeOff+L,8:11],o_,rd,1e30); dr=slab(nodes[nodeOff+R,4:7],nodes[nodeOff+R,8:11],o_,rd,1e30)
    N,F=(L,R) if not dl>dr else (R,L)
    vn,dn=walk(N,o_,d_,rd,np.float32(1e30))
    vf_ref,_=walk(F,o_,d_,rd,dn)
    vf_unc,_=walk(F,o_,d_,rd,np.float32(1e30))
    res.append((full,vn,vf_ref,vf_unc))
r=np.array(res); print('rays',len(r),'mean visits: full %.1f near %.1f far(ref) %.1f far(unculled) %.1f'%tuple(r.mean(0)))
print('max(near, far_unculled) mean %.1f'%np.maximum(r[:,1],r[:,3]).mean())

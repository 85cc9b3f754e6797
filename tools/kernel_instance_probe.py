import sys; sys.path.insert(0,'.')
import numpy as np, bench, bayesbridge_amd as bb
bb.set_verbose(0)
n,p=2000,6000
X=bench.make_columns(n,0,p); y,bt=bench.make_problem_y(n,p)
e=bb.Engine(bb.EngineConfig(n=n,p=p,seed=1,stream=0,trace_capacity=1),X,y); e.init_state(); e.run(1,5); e.sync()
print({ph: bb.kernel_instance(ph) for ph in ("lambda","gram","reduce","chol","solve","beta","eapply")})
e.set_state(bt,1.0,1.0,0.5); e.run(10,2); e.sync()
print({ph: bb.kernel_instance(ph) for ph in ("lambda","gram","reduce","chol","solve","beta","eapply")})

"""Debug: where does an fp8 gpt2-tiny resume diverge on the GPU (cache bytes, scale slots, params)?"""
import os, sys, tempfile
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from replicann_amd.training import TrainConfig, Trainer
from replicann_amd.ops.fp8 import fp8_states

kw = dict(model="gpt2-tiny", model_kwargs={"fp8": True}, batch_size=4, seq_len=128, steps=100,
          warmup_steps=1, lr=1e-3, log_every=10**9, seed=5, graph="off")
a = Trainer(TrainConfig(**kw))
for _ in range(3):
    a.step()
ck = os.path.join(tempfile.mkdtemp(), "c.pt")
a.save(ck)
qa = a.fp8_cache.qbuf.clone(); sa = [st.t.clone() for st in fp8_states(a.model)]; fa = a.flat.data.clone()
ra = [list(st.ready) for st in fp8_states(a.model)]
va = dict(a.fp8_cache.version)
b = Trainer(TrainConfig(**kw, resume=ck))
qb = b.fp8_cache.qbuf; sb = [st.t for st in fp8_states(b.model)]
print("flat equal", torch.equal(fa, b.flat.data))
print("qbuf equal", torch.equal(qa, qb), "refreshes a/b", a.fp8_cache.refreshes, b.fp8_cache.refreshes)
print("slots equal", [torch.equal(x, y) for x, y in zip(sa, sb)])
print("ready a", ra, "b", [list(st.ready) for st in fp8_states(b.model)])
print("versions b", len(b.fp8_cache.version), "a", len(va))
for x, y in zip(sa, sb):
    if not torch.equal(x, y):
        print(x.tolist(), y.tolist())
la = [float(a.step()) for _ in range(2)]
lb = [float(b.step()) for _ in range(2)]
print("losses", la, lb)

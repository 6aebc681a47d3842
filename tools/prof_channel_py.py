import cProfile, pstats, sys, os, time, torch
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "ad-federatedlearning_amd"))
import importlib
C = importlib.import_module("adfl_amd.Channel")
# python tools/prof_channel_py.py [SLQChannel|QSGDChannel|CNATChannel|...] (default SLQChannel)
CH = getattr(C, sys.argv[1] if len(sys.argv) > 1 else "SLQChannel")
base, rem = divmod(11_689_512, 256)
g = torch.Generator().manual_seed(0)
params = {}
for i in range(256):
    params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), generator=g) * 1e-3
    params[f"layer{i}.bias"] = torch.randn(64, generator=g) * 1e-3
ch = CH(4 if sys.argv[1:2] == ["PackedSLQChannel"] else 8)
for _ in range(5):
    qp, _ = ch.on_client_send(params); ch.on_server_receive(qp)
ts=[]
for _ in range(20):
    t=time.perf_counter(); qp,_=ch.on_client_send(params); t1=time.perf_counter(); ch.on_server_receive(qp); ts.append((t1-t, time.perf_counter()-t1))
print("enc min", min(a for a,_ in ts)*1e3, "dec min", min(b for _,b in ts)*1e3)
pr = cProfile.Profile(); pr.enable()
for _ in range(10):
    qp, _ = ch.on_client_send(params)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
pr = cProfile.Profile(); pr.enable()
for _ in range(10):
    ch.on_server_receive(qp)
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)

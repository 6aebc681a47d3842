import cProfile, pstats, sys, io
sys.argv=['x']
sys.path.insert(0, 'tools')
import torch
exec(open('tools/prof_channel_device.py').read().replace('if __name__ == "__main__":\n    main()', ''))
from adfl_amd.Channel import SLQChannel
dev = torch.device("cuda", 0)
base, rem = divmod(RESNET18, 256)
params = {}
for i in range(256):
    params[f"layer{i}.weight"] = torch.randn(1, base + (1 if i < rem else 0), device=dev) * 1e-3
    params[f"layer{i}.bias"] = torch.randn(64, device=dev) * 1e-3
ch = SLQChannel(8)
for _ in range(3):
    qp, _ = ch.on_client_send(params); ch.on_server_receive(qp)
pr = cProfile.Profile(); pr.enable()
for _ in range(10):
    qp, _ = ch.on_client_send(params); ch.on_server_receive(qp)
pr.disable()
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(18); print(s.getvalue()[:4000])

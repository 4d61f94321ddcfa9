"""FeaturesExtractor3D vs its float64 torch modules, conv1 forward in f32 and
in bf16x3 (rt_conv_set_precision): max feature error and per-parameter max
relative gradient error, and how many conv1 pooling windows pick another
argmax than float64 torch (r03 session 27)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import _rtpkg  # noqa: E402,F401
from ppo_radiotherapy_amd import _lib  # noqa: E402
from ppo_radiotherapy_amd.networks import FeaturesExtractor3D  # noqa: E402

out = {}
L = _lib.load()
for shape, B in [((4, 34, 27, 40), 6), ((4, 64, 64, 64), 2)]:
    for prec in ("f32", "bf16x3"):
        _lib.check(L.rt_conv_set_precision(_lib.CONV_PREC[prec]), "prec")
        torch.manual_seed(0)
        fe = FeaturesExtractor3D(shape, 64)
        ref = FeaturesExtractor3D(shape, 64).double()
        ref.load_state_dict({k: v.double() for k, v in fe.state_dict().items()})
        fe = fe.cuda()
        x = torch.rand((B, *shape))
        f = fe(x.cuda())
        fr = ref(x.double())
        gf = torch.randn_like(fr)
        f.backward(gf.float().cuda())
        fr.backward(gf)
        errs = {n: float((p.grad.cpu().double() - q.grad).abs().max()) / (float(q.grad.abs().max()) + 1e-12)
                for (n, p), q in zip(fe.named_parameters(), ref.parameters())}
        out[f"{shape[1]}x{shape[2]}x{shape[3]}_{prec}"] = {
            "feature_max_abs_err": float((f.detach().cpu().double() - fr).abs().max()),
            "grad_rel_err": errs}
        print(shape, prec, out[f"{shape[1]}x{shape[2]}x{shape[3]}_{prec}"]["feature_max_abs_err"],
              {k: round(v, 6) for k, v in errs.items() if "cnn" in k})
L.rt_conv_set_precision(0)
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "/dev/null", "w"), indent=1)

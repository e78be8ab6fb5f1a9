"""Shared decoding of the pooling golden cases (tests/golden/pool.npz, index 'pool'):
turns an index entry into the window arguments of hex pooling."""
from HyGrid import ops


def pool_args(m):
    """(method, kh, kw, sh, sw, hn, wn, pad, mode, value, ext_h, ext_w, ext_value)."""
    h, w = m["h"], m["w"]
    if m["kind"] == "pool":
        k, s = m["k"], m["s"]
        kh, kw = (k, k) if isinstance(k, int) else k
        sh, sw = (s, s) if isinstance(s, int) else s
        pl = ops.pool_plan(h, w, kh, kw, sh, sw, m["pad"], m.get("ceil", False),
                           m.get("cip", True))
        return (m["method"], kh, kw, sh, sw, pl["hn"], pl["wn"], m["pad"],
                m.get("mode", "constant"), m.get("value", 0), pl["ext_h"], pl["ext_w"],
                pl["ext_value"])
    if m["kind"] == "adaptive":
        hn = wn = m["outsize"]
        gh = int(h / hn)
        gw = int(w / (wn + 0.5)) if gh > 1 else int(w / wn)
        return (m["method"], gh, gw, gh, gw, hn, wn, 0, "constant", 0, 0, 0, 0.0)
    return (m["method"], h, w, h, w, 1, 1, 0, "constant", 0, 0, 0, 0.0)


def module_for(m):
    """The drop-in module a golden case exercises (HexFrames.py:255-410)."""
    from HyGrid import HexFrames as HF
    if m["kind"] == "pool":
        return HF.HexPool2d(m["method"], kernel_size=m["k"], stride=m["s"], padding=m["pad"],
                            padding_mode=m.get("mode", "constant"),
                            padding_value=m.get("value", 0), ceil_mode=m.get("ceil", False),
                            count_include_pad=m.get("cip", True))
    if m["kind"] == "adaptive":
        return HF.HexAdaptivePool2d(m["outsize"], m["method"])
    return HF.HexGlobalPool2d(m["method"])

"""The "mcprofile" renderer (MonteCarloProfileRenderer, src/renderers/mcprofile.cpp:443-586).

``MonteCarloProfileRenderer(...).render(ctx)`` traces the photons on the context's GPU
(mpss_mc_profile), computes the two multipole reference profiles (lerp on / off,
MultipoleReferenceTask, :381-425) on the host unless ``no_compare``, normalises, keeps
``result`` (MCProfileResult, mcprofile.h:52-68) and ``profile``, and writes the reference's
tab-separated file when ``filename`` is set: a header of ring-centre distances, six rows
(MC / Multipole / Lerped x Reflectance / Transmittance, each "name<TAB>total<TAB>values"), then
the same six rows multiplied by the distance (r * Rd(r)). Numbers print as an ostream at its
default precision (six significant digits, %g).

Photon streams: per-photon counter-based streams ("replay mode") rather than the
reference's per-task MT19937; the profile agrees with the reference's in distribution.
"""
import numpy as np

import mpss


def _g(x):
    return "%g" % x


class MonteCarloProfileRenderer:
    def __init__(self, layers, mfp_range=16.0, segments=1024, photons=100, filename="", no_compare=False,
                 seed=89):
        lay = np.asarray(layers, np.float32).reshape(-1, 4)
        if len(lay) < 1:
            raise ValueError("No layers param set for MCProfileRenderer.")
        self.layers = lay
        self.mfp_range = float(np.float32(mfp_range))
        self.segments = int(segments)
        self.photons = int(photons)
        self.filename = filename
        self.no_compare = no_compare
        self.seed = seed
        self.result = None
        self.profile = None

    def extent(self):
        """Render (:457-463): mfpRange x the mean over layers of 1 / (mua + musp)."""
        mfp = sum(1.0 / float(np.float32(a + b)) for a, b in self.layers[:, :2]) / len(self.layers)
        return self.mfp_range * mfp

    def render(self, ctx, stream=None):
        mc = ctx.mc_profile(self.layers, self.mfp_range, self.segments, self.photons, seed=self.seed, stream=stream)
        ref = {}
        if self.filename or not self.no_compare:
            for lerp in (False, True):
                ref[lerp] = mpss.mc_reference(self.layers, self.mfp_range, self.segments, lerp)
        self.profile = dict(reflectance=mc["reflectance"], transmittance=mc["transmittance"])
        self.result = dict(totalMCReflectance=mc["total_r"], totalMCTransmittance=mc["total_t"],
                           totalNoLerpReflectance=ref[False]["total_r"] if ref else 0.0,
                           totalNoLerpTransmittance=ref[False]["total_t"] if ref else 0.0,
                           totalLerpReflectance=ref[True]["total_r"] if ref else 0.0,
                           totalLerpTransmittance=ref[True]["total_t"] if ref else 0.0)
        self.reference = ref
        if self.filename:
            with open(self.filename, "w") as f:
                f.write(self.tsv())
        return self.result

    def tsv(self):
        """The output file of Render (:544-586)."""
        ext = self.extent()
        r = np.array([(i + .5) * ext / self.segments for i in range(self.segments)])
        res, ref = self.result, self.reference
        rows = [("Monte-Carlo Reflectance", res["totalMCReflectance"], self.profile["reflectance"]),
                ("Monte-Carlo Transmittance", res["totalMCTransmittance"], self.profile["transmittance"]),
                ("Multipole Reflectance", res["totalNoLerpReflectance"], ref[False]["reflectance"]),
                ("Multipole Transmittance", res["totalNoLerpTransmittance"], ref[False]["transmittance"]),
                ("Lerped Reflectance", res["totalLerpReflectance"], ref[True]["reflectance"]),
                ("Lerped Transmittance", res["totalLerpTransmittance"], ref[True]["transmittance"])]
        out = ["Name\tTotal" + "".join("\t" + _g(x) for x in r)]
        for mul in (None, r):
            for name, tot, vals in rows:
                v = vals if mul is None else vals * mul
                out.append(name + "\t" + _g(tot) + "\t" + "\t".join(_g(x) for x in v))
        return "\n".join(out) + "\n"


def create_from_params(ps):
    """CreateMonteCarloProfileRenderer (:609-625): layers, mfprange 16, segments 1024, photons
    "100" (a string), filename ""."""
    lay = ps.find("layers")
    if lay is None or len(lay) < 4:
        raise ValueError("No layers param set for MCProfileRenderer.")
    layers = [tuple(lay[4 * i:4 * i + 4]) for i in range(len(lay) // 4)]
    return MonteCarloProfileRenderer(layers, float(ps.one("mfprange", 16.0)), int(ps.one("segments", 1024)),
                                     int(str(ps.one("photons", "100"))), str(ps.one("filename", "")))


def read_tsv(path):
    """Parse a file written by ``tsv`` (or by the reference): distances and {row name: [(total,
    values), (total, r * values)]}."""
    with open(path) as f:
        lines = [l.rstrip("\n").split("\t") for l in f if l.strip()]
    dist = np.array([float(x) for x in lines[0][2:]])
    rows = {}
    for l in lines[1:]:
        rows.setdefault(l[0], []).append((float(l[1]), np.array([float(x) for x in l[2:]])))
    return dist, rows

"""Loader for the subset of pbrt-v2's scene language the multipole-skin path uses.

It mirrors the reference's parse-time API (core/api.cpp pbrtLookAt / pbrtCamera / pbrtShape /
pbrtMaterial / pbrtAreaLightSource / pbrtAttributeBegin ..., driven by core/pbrtparse.yy:771-796)
for the directives scenes/skin.pbrt and its relatives contain:

  Film "image" (xresolution, yresolution), LookAt, Camera "perspective" (fov, screenwindow),
  Sampler (pixelsamples), SurfaceIntegrator "multipolesubsurface" (maxdepth, maxerror,
  minsampledistance, mix, showirradiancepoints, incenter), WorldBegin/WorldEnd,
  AttributeBegin/End, TransformBegin/End, Translate, Rotate, Scale, Identity,
  Texture "constant" / "imagemap" (albedo, bumpmap), Material "layeredskin" (every parameter of
  CreateLayeredSkinMaterial, layeredskin.cpp:222-262, incl. genprofile / showirradiancepoints /
  irradiancepointsize / rgbprofile / usemontecarlo), AreaLightSource "area", LightSource "infinite"
  (L, scale, nsamples, mapname: .exr / .pfm / .tga via mpss.imageio), Shape "sphere" (as an area light only) and Shape "trianglemesh" (inline arrays, or "string npzfile" -- this
  package's stand-in for huge inline arrays, see tools/make_scene.py), Include.

Transforms follow core/transform.cpp (Translate, Scale, Rotate, LookAt, Perspective) evaluated in
float64 and rounded to float32 once; cameras/perspective.cpp + core/camera.cpp build
RasterToCamera.  Everything is handed to libmpss through the C ABI (mpss.Context).
"""
import math
import os
import re

import numpy as np

_TOKEN = re.compile(r'"[^"]*"|\[|\]|[^\s\[\]"]+')


def _tokens(text):
    for line in text.splitlines():
        # strip comments outside strings
        out, q = [], False
        for ch in line:
            if ch == '"':
                q = not q
            if ch == "#" and not q:
                break
            out.append(ch)
        for t in _TOKEN.findall("".join(out)):
            yield t


def _parse_value(tok):
    if tok.startswith('"'):
        return tok[1:-1]
    try:
        return float(tok) if any(c in tok for c in ".eE") else int(tok)
    except ValueError:
        return tok


class ParamSet(dict):
    """"type name" [values] pairs (core/paramset.h)."""

    def find(self, name, default=None):
        v = self.get(name)
        if v is None:
            return default
        return v[1]

    def one(self, name, default=None):
        v = self.find(name)
        return default if v is None else v[0]


def _read_params(toks, i):
    ps = ParamSet()
    while i < len(toks) and toks[i].startswith('"') and " " in toks[i].strip('"').strip():
        typ, name = toks[i][1:-1].split()
        i += 1
        if toks[i] == "[":
            j = toks.index("]", i)
            vals = [_parse_value(t) for t in toks[i + 1:j]]
            i = j + 1
        else:
            vals = [_parse_value(toks[i])]
            i += 1
        ps[name] = (typ, vals)
    return ps, i


# ------------------------------------------------------------------ transforms (core/transform.cpp)
def translate(d):
    m = np.eye(4)
    m[:3, 3] = d
    return m


def scale(s):
    return np.diag([s[0], s[1], s[2], 1.0])


def rotate(theta, axis):
    a = np.asarray(axis, np.float64)
    a = a / np.linalg.norm(a)
    s, c = math.sin(math.radians(theta)), math.cos(math.radians(theta))
    m = np.eye(4)
    m[0, 0] = a[0] * a[0] + (1 - a[0] * a[0]) * c
    m[0, 1] = a[0] * a[1] * (1 - c) - a[2] * s
    m[0, 2] = a[0] * a[2] * (1 - c) + a[1] * s
    m[1, 0] = a[0] * a[1] * (1 - c) + a[2] * s
    m[1, 1] = a[1] * a[1] + (1 - a[1] * a[1]) * c
    m[1, 2] = a[1] * a[2] * (1 - c) - a[0] * s
    m[2, 0] = a[0] * a[2] * (1 - c) - a[1] * s
    m[2, 1] = a[1] * a[2] * (1 - c) + a[0] * s
    m[2, 2] = a[2] * a[2] + (1 - a[2] * a[2]) * c
    return m


def look_at(pos, look, up):
    """World-to-camera of pbrt's LookAt (left-handed camera space, transform.cpp)."""
    pos, look, up = (np.asarray(v, np.float64) for v in (pos, look, up))
    d = look - pos
    d /= np.linalg.norm(d)
    u = up / np.linalg.norm(up)
    left = np.cross(u, d)
    left /= np.linalg.norm(left)
    new_up = np.cross(d, left)
    cam_to_world = np.eye(4)
    cam_to_world[:3, 0] = left
    cam_to_world[:3, 1] = new_up
    cam_to_world[:3, 2] = d
    cam_to_world[:3, 3] = pos
    return np.linalg.inv(cam_to_world)


def perspective(fov, n, f):
    persp = np.array([[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, f / (f - n), -f * n / (f - n)], [0, 0, 1, 0]],
                     np.float64)
    inv_tan = 1.0 / math.tan(math.radians(fov) / 2)
    return scale([inv_tan, inv_tan, 1]) @ persp


def camera_matrices(world_to_camera, fov, xres, yres, screen=None):
    """(RasterToCamera, CameraToWorld) of PerspectiveCamera (cameras/perspective.cpp:36-55,
    core/camera.cpp ProjectiveCamera ctor); fov applies to the shorter image axis."""
    frame = xres / yres
    if screen is None:
        screen = [-frame, frame, -1, 1] if frame > 1 else [-1, 1, -1 / frame, 1 / frame]
    if frame < 1:  # api.cpp MakeCamera: perspective fov is for the shorter axis
        pass
    cam_to_screen = perspective(fov, 1e-2, 1000.0)
    screen_to_raster = scale([xres, yres, 1]) @ scale([1 / (screen[1] - screen[0]), 1 / (screen[2] - screen[3]), 1]) \
        @ translate([-screen[0], -screen[3], 0])
    raster_to_camera = np.linalg.inv(cam_to_screen) @ np.linalg.inv(screen_to_raster)
    return raster_to_camera.astype(np.float32), np.linalg.inv(world_to_camera).astype(np.float32)


# ------------------------------------------------------------------ scene description
class Scene:
    def __init__(self):
        self.xres, self.yres = 640, 480
        self.fov = 90.0
        self.screen = None
        self.world_to_camera = np.eye(4)
        self.spp = 4
        self.integrator = {}
        self.materials = []  # list of layeredskin param dicts
        self.meshes = []     # dicts: P (world), N, S, uv, indices, o2w, w2o, reverse, material
        self.lights = []     # dicts: center, radius, L (rgb), nsamples; or kind="infinite", L, scale, l2w, w2l
        self.base_dir = "."
        self.renderer = None  # ("mcprofile", ParamSet) when the file selects the MC profile renderer

    def raster_to_camera(self):
        return camera_matrices(self.world_to_camera, self.fov, self.xres, self.yres, self.screen)


_SKIN_FLOATS = ("roughness", "nmperunit", "f_mel", "f_eu", "f_blood", "f_ohg", "ga_epi", "ga_derm", "b_derm")


def load(path, **override):
    sc = Scene()
    base = os.path.dirname(os.path.abspath(path))
    ctm = np.eye(4)
    state = dict(material=None, area=None, reverse=False)
    stack = []
    textures = {}
    in_world = False

    def run(text, base):
        nonlocal ctm, in_world, state
        toks = list(_tokens(text))
        i = 0
        while i < len(toks):
            d = toks[i]
            i += 1
            if d in ("WorldBegin",):
                in_world = True
                ctm = np.eye(4)
            elif d == "WorldEnd":
                pass
            elif d in ("AttributeBegin", "TransformBegin"):
                stack.append((ctm.copy(), dict(state)))
            elif d in ("AttributeEnd", "TransformEnd"):
                c, s = stack.pop()
                ctm = c
                if d == "AttributeEnd":
                    state = s
            elif d == "Identity":
                ctm = np.eye(4)
            elif d == "Translate":
                ctm = ctm @ translate([float(toks[i + k]) for k in range(3)])
                i += 3
            elif d == "Scale":
                ctm = ctm @ scale([float(toks[i + k]) for k in range(3)])
                i += 3
            elif d == "Rotate":
                ctm = ctm @ rotate(float(toks[i]), [float(toks[i + k]) for k in range(1, 4)])
                i += 4
            elif d == "LookAt":
                v = [float(toks[i + k]) for k in range(9)]
                ctm = ctm @ look_at(v[0:3], v[3:6], v[6:9])
                i += 9
            elif d == "ReverseOrientation":
                state["reverse"] = not state["reverse"]
            elif d == "Include":
                f = _parse_value(toks[i])
                i += 1
                fp = f if os.path.isabs(f) else os.path.join(base, f)
                run(open(fp).read(), os.path.dirname(fp))
            elif d in ("Film", "Camera", "Sampler", "SurfaceIntegrator", "VolumeIntegrator", "PixelFilter",
                       "Renderer", "Accelerator", "Material", "AreaLightSource", "Shape", "LightSource",
                       "Texture"):
                if d == "Texture":
                    name, _kind, cls = (_parse_value(toks[i + k]) for k in range(3))
                    i += 3
                else:
                    cls = _parse_value(toks[i])
                    i += 1
                ps, i = _read_params(toks, i)
                if d == "Film":
                    sc.xres = ps.one("xresolution", 640)
                    sc.yres = ps.one("yresolution", 480)
                elif d == "Camera":
                    if cls != "perspective":
                        raise ValueError("only the perspective camera is supported")
                    sc.fov = float(ps.one("fov", 90.0))
                    sc.screen = ps.find("screenwindow")
                    sc.world_to_camera = ctm.copy()
                elif d == "Sampler":
                    sc.spp = ps.one("pixelsamples", 4)
                elif d == "SurfaceIntegrator":
                    if cls != "multipolesubsurface":
                        raise ValueError("SurfaceIntegrator %r is outside this path" % cls)
                    sc.integrator = {k: v[1][0] for k, v in ps.items()}
                elif d == "Renderer":
                    if cls not in ("sampler", "mcprofile"):
                        raise ValueError("Renderer %r is outside this path" % cls)
                    sc.renderer = (cls, ps) if cls == "mcprofile" else None
                elif d in ("PixelFilter",):
                    if cls != "box" or ps.one("xwidth", 0.5) != 0.5 or ps.one("ywidth", 0.5) != 0.5:
                        raise ValueError("only the default 0.5-wide box filter is supported")
                elif d == "Texture":
                    textures[name] = _texture(cls, _kind, ps, base)
                elif d == "Material":
                    if cls != "layeredskin":
                        state["material"] = ("other", cls)
                    else:
                        state["material"] = ("layeredskin", _skin_params(ps, textures))
                elif d == "AreaLightSource":
                    state["area"] = (ps.find("L", [1.0, 1.0, 1.0]), ps.one("nsamples", 1))
                elif d == "LightSource":
                    if cls != "infinite":
                        raise ValueError("LightSource %r is outside this path" % cls)
                    mapname = ps.one("mapname", "")
                    if mapname:  # FindOneFilename: relative to the scene file's directory
                        mapname = mapname if os.path.isabs(mapname) else os.path.join(base, mapname)
                    sc.lights.append(dict(kind="infinite", L=_rgb3(ps.find("L", [1.0])), mapname=mapname or None,
                                          scale=_rgb3(ps.find("scale", [1.0])), nsamples=int(ps.one("nsamples", 1)),
                                          l2w=ctm.astype(np.float32), w2l=np.linalg.inv(ctm).astype(np.float32)))
                elif d == "Shape":
                    _shape(sc, cls, ps, ctm, state, base)
            else:
                raise ValueError("unsupported directive %r" % d)

    sc.base_dir = base
    run(open(path).read(), base)
    for k, v in override.items():
        setattr(sc, k, v)
    return sc


def _rgb3(v):
    v = list(v)
    return v * 3 if len(v) == 1 else v


def _texture(cls, typ, ps, base):
    """Texture "name" "color"|"spectrum"|"float" "constant"|"imagemap" (api.cpp pbrtTexture ->
    CreateConstant*Texture / CreateImage*Texture, textures/imagemap.cpp:110-180). An imagemap keeps
    the mpss.imagemap keywords; its file is read with mpss.imageio (FindFilename: relative to the
    scene file); a file that cannot be read gives the reference's one-valued map (texels None)."""
    if typ not in ("color", "spectrum", "float"):
        raise ValueError("texture type %r" % typ)
    if cls == "constant":
        return dict(cls="constant", type=typ, value=ps.find("value", [1.0]))
    if cls != "imagemap":
        raise ValueError("texture %r: only constant and imagemap textures are on this path (DESIGN.md)" % cls)
    mapping = ps.one("mapping", "uv")
    if mapping != "uv":
        raise ValueError("imagemap mapping %r: only the default uv mapping is on this path" % mapping)
    fn = ps.one("filename", "")
    path = fn if os.path.isabs(fn) else os.path.join(base, fn)
    texels = None
    if fn and os.path.exists(path):
        from mpss import imageio
        texels = imageio.read_image(path)
    else:
        import warnings
        warnings.warn("imagemap %r could not be read: one-valued texture (imagemap.cpp:76-81)" % fn)
    tex = dict(texels=texels, is_float=typ == "float", shift=float(ps.one("shift", 0.0)),
               scale=float(ps.one("scale", 1.0)), gamma=float(ps.one("gamma", 1.0)), wrap=ps.one("wrap", "repeat"),
               trilinear=ps.one("trilinear", "false") in ("true", True, 1),
               maxanisotropy=float(ps.one("maxanisotropy", 8.0)), uscale=float(ps.one("uscale", 1.0)),
               vscale=float(ps.one("vscale", 1.0)), udelta=float(ps.one("udelta", 0.0)),
               vdelta=float(ps.one("vdelta", 0.0)))
    return dict(cls="imagemap", type=typ, tex=tex, filename=fn)


def _skin_params(ps, textures):
    p = {}
    for k in _SKIN_FLOATS:
        if k in ps:
            p[k] = float(ps.one(k))
    lay = ps.find("layers")
    if lay is not None:
        p["layer_thickness_nm"] = [float(lay[0]), float(lay[2])]
        p["layer_ior"] = [float(lay[1]), float(lay[3])]
    for k in ("Kr", "Kt", "albedo"):
        if k in ps:
            typ, vals = ps[k]
            if typ == "texture":
                if vals[0] not in textures:
                    raise ValueError("texture %r is not defined" % vals[0])
                t = textures[vals[0]]
                if t["type"] == "float":
                    raise ValueError("%s needs a spectrum texture, %r is a float texture" % (k, vals[0]))
                if t["cls"] == "imagemap":
                    if k != "albedo":
                        raise ValueError("an imagemap %s is outside this path (DESIGN.md); albedo and bumpmap "
                                         "take image textures" % k)
                    p["albedo_tex"] = t["tex"]
                    continue
                vals = t["value"]
            p[k] = _rgb3(vals)
    if "bumpmap" in ps:
        typ, vals = ps["bumpmap"]
        t = textures.get(vals[0]) if typ == "texture" else None
        if t is None or t["cls"] != "imagemap" or t["type"] != "float":
            raise ValueError("bumpmap: only a float imagemap texture is on this path")
        p["bump_tex"] = t["tex"]
    for k in ("desiredlength",):
        if k in ps:
            p["desired_length"] = int(ps.one(k))
    if "irradiancepointsize" in ps:
        p["irradiance_point_size"] = float(ps.one("irradiancepointsize"))
    if "photons" in ps:  # a string parameter parsed with _strtoui64 (layeredskin.cpp:251-252)
        p["photons"] = int(str(ps.one("photons")))
    for k, dst in (("lerponthinslab", "lerp_on_thin_slab"), ("doublerefsslf", "double_ref_sslf"),
                   ("usemontecarlo", "use_monte_carlo"), ("rgbprofile", "rgb_profile"), ("genprofile", "gen_profile"),
                   ("showirradiancepoints", "show_irradiance_points")):
        if k in ps:
            v = ps.one(k)
            p[dst] = int(v in (True, "true", 1))
    if p.get("gen_profile", 1) == 0:
        import warnings
        warnings.warn("LayeredSkin genprofile false: no Mo() term on this material (the reference would dereference "
                      "its NULL MultipoleBSSRDFData, layeredskin.cpp:184; DESIGN.md section 2)")
    return p


def _shape(sc, cls, ps, ctm, state, base):
    if cls == "sphere":
        if state["area"] is None:
            raise ValueError("a sphere is supported only as an area light's shape")
        r = float(ps.one("radius", 1.0))
        lin = ctm[:3, :3]
        if not np.allclose(lin, np.eye(3)):
            raise ValueError("area-light spheres may only be translated")
        sc.lights.append(dict(center=ctm[:3, 3].astype(np.float32), radius=r, L=_rgb3(state["area"][0]),
                              nsamples=int(state["area"][1])))
        return
    if cls != "trianglemesh":
        raise ValueError("shape %r is outside this path" % cls)
    if state["area"] is not None:
        raise ValueError("emissive triangle meshes are outside this path")
    if "npzfile" in ps:
        f = ps.one("npzfile")
        z = np.load(f if os.path.isabs(f) else os.path.join(base, f), allow_pickle=False)
        arr = {k: z[k] for k in z.files}
    else:
        arr = {k: np.asarray(ps.find(k)) for k in ("P", "N", "S", "uv", "indices") if k in ps}
        if "st" in ps:
            arr["uv"] = np.asarray(ps.find("st"))
    if state["material"] is None or state["material"][0] != "layeredskin":
        raise ValueError("meshes need a layeredskin material on this path")
    mat = state["material"][1]
    if not any(x is mat for x in sc.materials):  # one material per Material directive
        sc.materials.append(mat)
    o2w = ctm
    P = np.asarray(arr["P"], np.float32).reshape(-1, 3).astype(np.float64)
    Pw = (P @ o2w[:3, :3].T + o2w[:3, 3]).astype(np.float32)  # TriangleMesh ctor: (*ObjectToWorld)(P[i])
    sc.meshes.append(dict(P=Pw, N=arr.get("N"), S=arr.get("S"), uv=arr.get("uv"),
                          indices=np.asarray(arr["indices"], np.int32).reshape(-1, 3),
                          o2w=o2w.astype(np.float32), w2o=np.linalg.inv(o2w).astype(np.float32),
                          reverse=state["reverse"],
                          material=next(i for i, x in enumerate(sc.materials) if x is mat)))


def subdivide_mesh(me, levels):
    """Midpoint (1:4) subdivision of a loaded trianglemesh dict, `levels` times: the same surface
    with 4^levels as many triangles (BASELINE.json config C5's synthetic dense head). N and S are
    interpolated and renormalised, uv interpolated; winding is kept."""
    P = np.asarray(me["P"], np.float64)
    idx = np.asarray(me["indices"], np.int64)
    att = {k: (None if me.get(k) is None else np.asarray(me[k], np.float64)) for k in ("N", "S", "uv")}
    for _ in range(levels):
        a, b, c = idx[:, 0], idx[:, 1], idx[:, 2]
        e = np.concatenate([np.stack([a, b], 1), np.stack([b, c], 1), np.stack([c, a], 1)])
        key = np.sort(e, 1)
        uniq, inv = np.unique(key, axis=0, return_inverse=True)
        inv = inv.reshape(-1)
        base = len(P)
        P = np.concatenate([P, 0.5 * (P[uniq[:, 0]] + P[uniq[:, 1]])])
        for k, v in att.items():
            if v is None:
                continue
            m = 0.5 * (v[uniq[:, 0]] + v[uniq[:, 1]])
            if k in ("N", "S"):
                m /= np.maximum(np.linalg.norm(m, axis=1, keepdims=True), 1e-20)
            att[k] = np.concatenate([v, m])
        nt = len(idx)
        ab, bc, ca = base + inv[:nt], base + inv[nt:2 * nt], base + inv[2 * nt:]
        idx = np.concatenate([np.stack([a, ab, ca], 1), np.stack([ab, b, bc], 1), np.stack([ca, bc, c], 1),
                              np.stack([ab, bc, ca], 1)])
    out = dict(me)
    out["P"] = P.astype(np.float32)
    out["indices"] = idx.astype(np.int32)
    for k, v in att.items():
        out[k] = None if v is None else v.astype(np.float32)
    return out


def mesh_points(sc, min_dist=None):
    """SurfacePoints of a scene's meshes by the product's host tessellator (the pointsfile a
    TessellateSurfacePointsRenderer pass would write), e.g. to pair a subdivided mesh with the
    points of the original surface."""
    import mpss
    md = float(sc.integrator.get("minsampledistance", 0.25)) if min_dist is None else min_dist
    parts = []
    for me in sc.meshes:
        det = np.linalg.det(np.asarray(me["o2w"], np.float64)[:3, :3])
        parts.append(mpss.host_tessellate(me["P"], me["indices"], me["o2w"], me["w2o"], md, N=me["N"], S=me["S"],
                                          uv=me["uv"], flip=bool(me["reverse"]) ^ bool(det < 0),
                                          material=me["material"]))
    return np.concatenate(parts)


def integrator_config(sc, **kw):
    """mpss_config from the SurfaceIntegrator line (CreateMultipoleSubsurfaceIntegrator)."""
    it = sc.integrator
    cfg = dict(max_depth=int(it.get("maxdepth", 5)), max_error=float(it.get("maxerror", 0.05)),
               min_sample_distance=float(it.get("minsampledistance", 0.25)), mix=float(it.get("mix", 0.5)),
               show_irradiance_points=int(it.get("showirradiancepoints", "false") == "true"),
               incenter=int(it.get("incenter", "false") == "true"),
               use_poisson_point_finder=int(it.get("usepoissonpointfinder", "false") in ("true", True, 1)))
    cfg.update(kw)
    return cfg


def infinite_L(li):
    """CreateInfiniteLight's L * scale (lights/infinite.cpp:180-188): both "color" parameters are
    Spectrum::FromRGB (reflectance, paramset.cpp:97-105), multiplied band by band."""
    import mpss
    return (mpss.host_from_rgb(li["L"]) * mpss.host_from_rgb(li["scale"])).astype(np.float32)


def infinite_texels(li):
    """The light's map as ReadImage returns it (mpss.imageio), or None without "mapname";
    "texels" in the dict (an (H, W, 3) array) overrides the file."""
    if li.get("texels") is not None:
        return np.ascontiguousarray(li["texels"], np.float32)
    if not li.get("mapname"):
        return None
    from mpss import imageio
    return imageio.read_image(li["mapname"])


def build_context(sc, **cfg_kw):
    """Create an mpss.Context holding the scene (materials, meshes, lights, camera)."""
    import mpss
    ctx = mpss.Context(**integrator_config(sc, **cfg_kw))
    mids = []
    for m in sc.materials:
        kw = {k: v for k, v in m.items() if k not in ("Kr", "Kt", "albedo", "albedo_tex", "bump_tex")}
        for k in ("Kr", "Kt", "albedo"):
            if k in m:
                kw[k] = mpss.host_from_rgb(m[k])
        mids.append(ctx.add_layeredskin(mpss.default_skin(**kw)))
    for m, mid in zip(sc.materials, mids):
        if m.get("albedo_tex") is not None or m.get("bump_tex") is not None:
            alb = ctx.add_imagemap(**m["albedo_tex"]) if m.get("albedo_tex") is not None else -1
            bump = ctx.add_imagemap(**m["bump_tex"]) if m.get("bump_tex") is not None else -1
            ctx.set_material_textures(mid, alb, bump)
    for me in sc.meshes:
        ctx.add_mesh(me["P"], me["indices"], me["o2w"], me["w2o"], mids[me["material"]], N=me["N"], S=me["S"],
                     uv=me["uv"], reverse=me["reverse"])
    for li in sc.lights:
        if li.get("kind") == "infinite":
            ctx.add_infinite_light(infinite_L(li), li["nsamples"], li["l2w"], li["w2l"], texels=infinite_texels(li))
        else:
            ctx.add_sphere_light(li["center"], li["radius"], mpss.host_from_rgb(li["L"]), li["nsamples"])
    r2c, c2w = sc.raster_to_camera()
    ctx.set_camera(r2c, c2w, sc.xres, sc.yres)
    pf = sc.integrator.get("pointsfile")
    if pf:  # MultipoleSubsurfaceIntegrator reads the points instead of tessellating
        ctx.load_pointsfile(pf if os.path.isabs(pf) else os.path.join(sc.base_dir, pf))
    return ctx

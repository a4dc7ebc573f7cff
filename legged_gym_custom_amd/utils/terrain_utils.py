"""Sub-terrain height-field generators — drop-in for legged_gym/utils/terrain_utils.py.

Host-side, setup-time numpy (the reference builds the terrain on the CPU too). Every
generator reproduces the reference's int16 output bit for bit: the same unit
conversions (`int()` truncation or Python `round()`, as the reference uses at each
site), the same numpy RNG calls in the same order (so a run seeded with
`np.random.seed(s)` draws the same tiles), and the same float expression order wherever
a float is truncated to int16. Pinned by tests/test_terrain.py against fixtures made by
tools/gen_terrain_golden.py from the reference itself.

Layout (terrain_utils.py:467-476): `height_field_raw[length, width]`, rows = x (along
the course), cols = y; heights in units of `vertical_scale`.

One restated dependency: `random_uniform_terrain` upsamples with `scipy.interpolate.
interp2d(kind='linear')` (terrain_utils.py:42), removed in SciPy 1.14. On a rectilinear
grid that call is an exact tensor-product linear spline, i.e. bilinear interpolation;
`_bilinear_upsample` restates it.
"""
import numpy as np


class SubTerrain:
    """terrain_utils.py:467-476: one tile, `height_field_raw` int16 [length, width]."""

    def __init__(self, terrain_name="terrain", width=256, length=256, vertical_scale=1.0, horizontal_scale=1.0):
        self.terrain_name = terrain_name
        self.vertical_scale = vertical_scale
        self.horizontal_scale = horizontal_scale
        self.width = width
        self.length = length
        self.height_field_raw = np.zeros((self.length, self.width), dtype=np.int16)


def _bilinear_upsample(coarse, rows_in, cols_in, rows_out, cols_out):
    """Bilinear interpolation of `coarse[len(rows_in), len(cols_in)]` (ascending grids) at
    the grid rows_out x cols_out — the value interp2d(kind='linear') returns there."""
    def axis(src, dst):
        i = np.clip(np.searchsorted(src, dst, side="right") - 1, 0, len(src) - 2)
        t = (dst - src[i]) / (src[i + 1] - src[i])
        return i, np.clip(t, 0.0, 1.0)

    ri, rt = axis(rows_in, rows_out)
    ci, ct = axis(cols_in, cols_out)
    z = coarse.astype(np.float64)
    top = z[ri][:, ci] * (1.0 - ct)[None, :] + z[ri][:, ci + 1] * ct[None, :]
    bot = z[ri + 1][:, ci] * (1.0 - ct)[None, :] + z[ri + 1][:, ci + 1] * ct[None, :]
    return top * (1.0 - rt)[:, None] + bot * rt[:, None]


def random_uniform_terrain(terrain, min_height, max_height, step=1, downsampled_scale=None):
    """terrain_utils.py:9-51: uniform random heights on a coarse grid (one
    np.random.choice draw of the whole grid), bilinearly upsampled, rounded, added."""
    if downsampled_scale is None:
        downsampled_scale = terrain.horizontal_scale
    vs, hs = terrain.vertical_scale, terrain.horizontal_scale
    lo, hi, st = int(min_height / vs), int(max_height / vs), int(step / vs)
    levels = np.arange(lo, hi + st, st)
    n_r = int(terrain.length * hs / downsampled_scale)
    n_c = int(terrain.width * hs / downsampled_scale)
    coarse = np.random.choice(levels, (n_r, n_c))
    fine = _bilinear_upsample(coarse,
                              np.linspace(0, terrain.length * hs, n_r), np.linspace(0, terrain.width * hs, n_c),
                              np.linspace(0, terrain.length * hs, terrain.length),
                              np.linspace(0, terrain.width * hs, terrain.width))
    terrain.height_field_raw += np.rint(fine).astype(np.int16)
    return terrain


def sloped_terrain(terrain, slope=1):
    """terrain_utils.py:53-68: a ramp across the width (columns)."""
    _, w = terrain.height_field_raw.shape
    top = int(slope * (terrain.horizontal_scale / terrain.vertical_scale) * w)
    ramp = (np.arange(w) / (w - 1)) * top
    terrain.height_field_raw += ramp.astype(terrain.height_field_raw.dtype)[None, :]
    return terrain


def pyramid_sloped_terrain(terrain, slope=1, platform_size=1.0):
    """terrain_utils.py:70-89 (this fork's version): height max_h * fx * fy with fx, fy
    the normalised distance-to-edge along each axis, clipped to the value at the
    platform corner (a flat top of side `platform_size`)."""
    hf = terrain.height_field_raw
    n_l, n_w = hf.shape
    cx, cy = n_w // 2, n_l // 2
    fx = (cx - np.abs(np.arange(n_w) - cx)) / cx
    fy = (cy - np.abs(np.arange(n_l) - cy)) / cy
    fyy, fxx = np.meshgrid(fy, fx, indexing="ij")
    top = int(slope * (terrain.horizontal_scale / terrain.vertical_scale) * (n_w / 2))
    hf += (top * fxx * fyy).astype(hf.dtype)
    half = int(platform_size / terrain.horizontal_scale / 2)
    corner = hf[cy - half, cx - half]
    terrain.height_field_raw = np.clip(hf, min(corner, 0), max(corner, 0))
    return terrain


def discrete_obstacles_terrain(terrain, max_height, min_size, max_size, num_rects, platform_size=1.0):
    """terrain_utils.py:91-117: num_rects random rectangles (sizes/corners on a 4-cell
    lattice) at one of {-h, -h/2, h/2, h}, then a cleared central platform."""
    hf = terrain.height_field_raw
    h = int(max_height / terrain.vertical_scale)
    s_lo = int(min_size / terrain.horizontal_scale)
    s_hi = int(max_size / terrain.horizontal_scale)
    plat = int(platform_size / terrain.horizontal_scale)
    n_l, n_w = hf.shape
    levels = [-h, (-h) // 2, h // 2, h]
    for _ in range(num_rects):
        rw = np.random.choice(range(s_lo, s_hi, 4))
        rl = np.random.choice(range(s_lo, s_hi, 4))
        r0 = np.random.choice(range(0, n_l - rl, 4))
        c0 = np.random.choice(range(0, n_w - rw, 4))
        hf[r0:r0 + rl, c0:c0 + rw] = np.random.choice(levels)
    hf[(n_l - plat) // 2:(n_l + plat) // 2, (n_w - plat) // 2:(n_w + plat) // 2] = 0
    return terrain


def wave_terrain(terrain, num_waves=1, amplitude=1.0):
    """terrain_utils.py:119-132: amp * (cos(row / dy) + sin(col / dx))."""
    amp = int(0.5 * amplitude / terrain.vertical_scale)
    if num_waves <= 0:
        return terrain
    n_l, n_w = terrain.height_field_raw.shape
    dy = n_l / (num_waves * 2 * np.pi)
    dx = n_w / (num_waves * 2 * np.pi)
    rr, cc = np.meshgrid(np.arange(n_l), np.arange(n_w), indexing="ij")
    terrain.height_field_raw += (amp * (np.cos(rr / dy) + np.sin(cc / dx))).astype(terrain.height_field_raw.dtype)
    return terrain


def stairs_terrain(terrain, step_width, step_height):
    """terrain_utils.py:134-147: steps rising along the rows."""
    sw = int(step_width / terrain.horizontal_scale)
    sh = int(step_height / terrain.vertical_scale)
    n_l = terrain.height_field_raw.shape[0]
    for k in range(n_l // sw):
        terrain.height_field_raw[k * sw:(k + 1) * sw, :] += sh * (k + 1)
    return terrain


def pyramid_stairs_terrain(terrain, step_width, step_height, platform_size=1.0):
    """terrain_utils.py:149-164: concentric rings, each one step higher, until the
    remaining square is no wider than the platform."""
    sw = int(step_width / terrain.horizontal_scale)
    sh = int(step_height / terrain.vertical_scale)
    plat = int(platform_size / terrain.horizontal_scale)
    n_l, n_w = terrain.height_field_raw.shape
    r0, r1, c0, c1, level = 0, n_l, 0, n_w, 0
    while r1 - r0 > plat and c1 - c0 > plat:
        r0, r1, c0, c1 = r0 + sw, r1 - sw, c0 + sw, c1 - sw
        level += sh
        terrain.height_field_raw[r0:r1, c0:c1] = level
    return terrain


def stepping_stones_terrain(terrain, stone_size, stone_distance, max_height, platform_size=1., depth=-10):
    """terrain_utils.py:166-212: pit everywhere, then rows of stones (random phase per
    row, random height per stone), then a cleared central platform."""
    hf = terrain.height_field_raw
    size = int(stone_size / terrain.horizontal_scale)
    gap = int(stone_distance / terrain.horizontal_scale)
    h = int(max_height / terrain.vertical_scale)
    plat = int(platform_size / terrain.horizontal_scale)
    pit = int(depth / terrain.vertical_scale)
    n_l, n_w = hf.shape
    hf[:] = pit
    levels = np.arange(-h - 1, h, 1)
    r = 0
    while r < n_l:
        r_end = min(n_l, r + size)
        c = np.random.randint(0, size)
        hf[r:r_end, 0:max(0, c - gap)] = np.random.choice(levels)
        while c < n_w:
            hf[r:r_end, c:min(n_w, c + size)] = np.random.choice(levels)
            c += size + gap
        r += size + gap
    hf[(n_l - plat) // 2:(n_l + plat) // 2, (n_w - plat) // 2:(n_w + plat) // 2] = 0
    return terrain


def _perimeter_walls(hf, cells, height, front_back):
    """Side walls (min/max column); front/back walls too when asked. `cells` == 0
    keeps numpy's `[-0:]` meaning (the whole axis), as the reference's slicing does."""
    hf[:, :cells] = height
    hf[:, -cells:] = height
    if front_back:
        hf[:cells, :] = height
        hf[-cells:, :] = height


def parkour_hurdle_terrain_randomized(terrain, platform_len=2.5, platform_height=0.5, x_range=(14.0, 14.1),
                                      y_range=(-6.0, -5.9), num_hurdles=1, hurdle_thickness=0.3,
                                      hurdle_height_range=(0.2, 0.3), half_valid_width=(2.4, 2.5), border_width=0.1,
                                      border_height=0.5):
    """terrain_utils.py:215-310: a start platform, then hurdles at random spacing whose
    bars are cut down to 0 outside a corridor of random half-width; perimeter walls.
    `terrain.hurdles` lists the hurdle (x, y) in tile coordinates."""
    hs, vs = terrain.horizontal_scale, terrain.vertical_scale
    hf = terrain.height_field_raw
    terrain.hurdles = []
    mid = terrain.width // 2
    x_lo, x_hi = round(x_range[0] / hs), round(x_range[1] / hs)
    y_lo, y_hi = round(y_range[0] / hs), round(y_range[1] / hs)
    half = round(np.random.uniform(half_valid_width[0], half_valid_width[1]) / hs)
    h_lo, h_hi = round(hurdle_height_range[0] / vs), round(hurdle_height_range[1] / vs)
    plat = round(platform_len / hs)
    hf[:plat, :] = round(platform_height / vs)
    bar = round(hurdle_thickness / hs)
    x = plat
    for _ in range(num_hurdles):
        x += np.random.randint(x_lo, x_hi)
        dy = np.random.randint(y_lo, y_hi)
        h = np.random.randint(h_lo, h_hi)
        a, b = x - bar // 2, x + bar // 2
        hf[a:b, :] = h
        hf[a:b, :mid + dy - half] = 0
        hf[a:b, mid + dy + half:] = 0
        terrain.hurdles.append((x * hs, (mid + dy) * hs))
    np.random.randint(x_lo, x_hi)  # the final-platform draw (terrain_utils.py:294), result unused
    _perimeter_walls(hf, int(border_width / hs), int(border_height / vs), front_back=True)


def parkour_terrain(terrain, start_platform_length=2.5, start_platform_height=0.5, x_positions=(7.0, 11.0, 14.5),
                    y_positions=(0.0, 0.0, 0.0), obstacle_lengths=(0.5, 0.5, 0.5), obstacle_heights=None,
                    half_valid_width=2.5, border_width=0.1, border_height=0.5):
    """terrain_utils.py:312-380: obstacles (bars of the given length/height; negative
    heights are gaps) at exact (x, y) positions inside a corridor of half-width
    `half_valid_width` around the course midline, after a start platform; side walls
    only (the robot enters and leaves through the tile ends)."""
    n = len(x_positions)
    assert len(y_positions) == n, "x_positions and y_positions must have the same length"
    assert len(obstacle_lengths) == n, "hurdle_thickness must have num_hurdles elements"
    if obstacle_heights is not None:
        assert len(obstacle_heights) == n, "hurdle_heights must have same length as x_positions"
    hs, vs = terrain.horizontal_scale, terrain.vertical_scale
    hf = terrain.height_field_raw
    terrain.hurdle_positions = []
    mid = terrain.width // 2
    hf[:round(start_platform_length / hs), :] = round(start_platform_height / vs)
    half = round(half_valid_width / hs)
    for xm, ym, ln, ht in zip(x_positions, y_positions, obstacle_lengths,
                              obstacle_heights if obstacle_heights is not None else [None] * n):
        cx, cy = round(xm / hs), mid + round(ym / hs)
        h = round(ht / vs)  # (a None height fails here, as in the reference)
        bar = round(ln / hs)
        a, b = cx - bar // 2, cx + bar // 2
        hf[a:b, :] = h
        hf[a:b, :cy - half] = 0
        hf[a:b, cy + half:] = 0
        terrain.hurdle_positions.append((xm, ym))
    _perimeter_walls(hf, int(border_width / hs), int(border_height / vs), front_back=False)


def slope_moves(hf, threshold_cells):
    """Per-vertex x/y shift (in cells, each in {-1, 0, 1}) that turns steps steeper than
    the threshold into vertical walls (terrain_utils.py:401-446): a vertex moves
    toward a neighbour that is more than `threshold_cells` higher; the diagonal
    neighbour is used only on an axis the direct neighbours left unmoved."""
    r, c = hf.shape  # differences in the field's own dtype (int16), as the reference takes them
    mx = np.zeros((r, c))
    my = np.zeros((r, c))
    md = np.zeros((r, c))
    mx[:r - 1, :] += hf[1:, :] - hf[:r - 1, :] > threshold_cells
    mx[1:, :] -= hf[:r - 1, :] - hf[1:, :] > threshold_cells
    my[:, :c - 1] += hf[:, 1:] - hf[:, :c - 1] > threshold_cells
    my[:, 1:] -= hf[:, :c - 1] - hf[:, 1:] > threshold_cells
    md[:r - 1, :c - 1] += hf[1:, 1:] - hf[:r - 1, :c - 1] > threshold_cells
    md[1:, 1:] -= hf[:r - 1, :c - 1] - hf[1:, 1:] > threshold_cells
    return mx + md * (mx == 0), my + md * (my == 0)


def convert_heightfield_to_trimesh(height_field_raw, horizontal_scale, vertical_scale, slope_threshold=None):
    """terrain_utils.py:382-465: vertices [rows*cols, 3] float32 (row-major grid, x along
    rows) and triangles [2*(rows-1)*(cols-1), 3] uint32, two per cell:
    (v00, v11, v01) and (v00, v10, v11)."""
    hf = height_field_raw
    n_r, n_c = hf.shape
    gx = np.linspace(0, (n_r - 1) * horizontal_scale, n_r)
    gy = np.linspace(0, (n_c - 1) * horizontal_scale, n_c)
    yy, xx = np.meshgrid(gy, gx)
    if slope_threshold is not None:
        dx, dy = slope_moves(hf, slope_threshold * (horizontal_scale / vertical_scale))
        xx = xx + dx * horizontal_scale
        yy = yy + dy * horizontal_scale
    vertices = np.empty((n_r * n_c, 3), dtype=np.float32)
    vertices[:, 0] = xx.reshape(-1)
    vertices[:, 1] = yy.reshape(-1)
    vertices[:, 2] = hf.reshape(-1) * vertical_scale
    v00 = (np.arange(n_r - 1)[:, None] * n_c + np.arange(n_c - 1)[None, :]).reshape(-1).astype(np.uint32)
    tri = np.empty((v00.size, 2, 3), dtype=np.uint32)
    tri[:, 0, 0], tri[:, 0, 1], tri[:, 0, 2] = v00, v00 + n_c + 1, v00 + 1
    tri[:, 1, 0], tri[:, 1, 1], tri[:, 1, 2] = v00, v00 + n_c, v00 + n_c + 1
    return vertices, tri.reshape(-1, 3)


def pack_mesh(height_field_raw, horizontal_scale, vertical_scale, slope_threshold=None):
    """The collision surface the step kernel reads (lgx_buffers.terrain_mesh): one uint32
    per vertex = int16 height | (dx + 1) << 16 | (dy + 1) << 18, where (dx, dy) is the
    slope-threshold wall shift of convert_heightfield_to_trimesh (zero without a
    threshold, i.e. a PhysX-style heightfield). 4 B/vertex instead of the reference's
    12 B vertex + 24 B of triangle indices; the mesh is rebuilt on the fly per query."""
    hf = height_field_raw
    word = hf.astype(np.int16).view(np.uint16).astype(np.uint32)
    if slope_threshold is None:
        dx = dy = np.zeros(hf.shape)
    else:
        dx, dy = slope_moves(hf, slope_threshold * (horizontal_scale / vertical_scale))
    word |= (dx + 1).astype(np.uint32) << np.uint32(16)
    word |= (dy + 1).astype(np.uint32) << np.uint32(18)
    return word | mesh_block_bits(hf)


MESH_BLOCK = 8  # lgx_env.hip MESH_BLOCK


def mesh_block_bits(hf, block=MESH_BLOCK):
    """Bits 20-31 of every mesh word: a conservative maximum height of the vertex's 8 x 8 block
    (bits 20-30: q = ceil((max + 32768) / 32), decoded as 32 q - 32768 >= max; bit 31: present —
    absent when q would not fit 11 bits). The kernel's contact query skips spheres above every
    vertex their cell range can reach (lgx_env.hip terrain_contact_wave)."""
    h = hf.astype(np.int64)
    R, C = h.shape
    pr, pc = -R % block, -C % block
    hp = np.pad(h, ((0, pr), (0, pc)), constant_values=np.iinfo(np.int16).min)
    bm = hp.reshape((R + pr) // block, block, (C + pc) // block, block).max(axis=(1, 3))
    q = -((-(bm + 32768)) // 32)  # ceil
    ok = q <= 2047
    bits = np.where(ok, (q.clip(0, 2047).astype(np.uint32) << np.uint32(20)) | np.uint32(1 << 31), np.uint32(0))
    return np.repeat(np.repeat(bits, block, axis=0), block, axis=1)[:R, :C].astype(np.uint32)

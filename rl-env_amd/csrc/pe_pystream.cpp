// pe_pystream.cpp -- seed-exact reset maps: the reference's _generate_map
// (plantos_env.py:338-372) driven by CPython's global `random` stream, on the host.
//
// The reference draws every layout from CPython's module-level Mersenne Twister
// (the reset seed is ignored, plantos_env.py:127 vs 344-372) and its candidate
// lists come from iterating Python sets of (x, y) tuples, so a seed-exact layout
// needs (SURVEY.md §7 hard part 1):
//   * MT19937 with random.seed(int) seeding (init_by_array over the 32-bit
//     chunks of abs(seed)), getrandbits(k <= 32), _randbelow_with_getrandbits,
//     random() (53 bits), randint / choice / sample (CPython 3.10 random.py);
//   * the iteration order of CPython 3.10 sets (Objects/setobject.c: open
//     addressing, LINEAR_PROBES = 9, PERTURB_SHIFT = 5, resize rules,
//     set_difference's copy-and-discard vs rebuild paths) over tuple hashes
//     (Objects/tupleobject.c xxHash mix; hash(small int) = int).
// Maps come out in stream order; the vec-env assigns them to envs the way
// DummyVecEnv consumes them (env-index order at reset, then per step).
// C-ABI: pe_pystream_* in include/plantos_batch.h.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/plantos_batch.h"

extern "C" int pe_internal_set_error(int code, const char* msg);

namespace {

// ---------------------------------------------------------------- MT19937
struct Mt {
  uint32_t s[624];
  int i = 625;

  void init_genrand(uint32_t v) {
    s[0] = v;
    for (int k = 1; k < 624; ++k) s[k] = 1812433253u * (s[k - 1] ^ (s[k - 1] >> 30)) + (uint32_t)k;
    i = 624;
  }
  // random.seed(int): init_by_array over abs(seed) in 32-bit little-endian chunks
  void seed(uint64_t a) {
    uint32_t key[2] = {(uint32_t)a, (uint32_t)(a >> 32)};
    const int len = key[1] ? 2 : 1;
    init_genrand(19650218u);
    int k = 1, j = 0;
    for (int n = 624 > len ? 624 : len; n; --n) {
      s[k] = (s[k] ^ ((s[k - 1] ^ (s[k - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
      if (++k >= 624) {
        s[0] = s[623];
        k = 1;
      }
      if (++j >= len) j = 0;
    }
    for (int n = 623; n; --n) {
      s[k] = (s[k] ^ ((s[k - 1] ^ (s[k - 1] >> 30)) * 1566083941u)) - (uint32_t)k;
      if (++k >= 624) {
        s[0] = s[623];
        k = 1;
      }
    }
    s[0] = 0x80000000u;
    i = 624;
  }
  uint32_t next() {
    if (i >= 624) {
      for (int k = 0; k < 624; ++k) {
        const uint32_t y = (s[k] & 0x80000000u) | (s[(k + 1) % 624] & 0x7fffffffu);
        s[k] = s[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      i = 0;
    }
    uint32_t y = s[i++];
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
  }
  uint32_t getrandbits(int k) { return next() >> (32 - k); }  // 1 <= k <= 32
  // random.py _randbelow_with_getrandbits
  uint32_t below(uint32_t n) {
    if (!n) return 0;
    int k = 0;
    for (uint32_t t = n; t; t >>= 1) ++k;  // n.bit_length()
    uint32_t r = getrandbits(k);
    while (r >= n) r = getrandbits(k);
    return r;
  }
  double random() {
    const uint32_t a = next() >> 5, b = next() >> 6;
    return ((double)a * 67108864.0 + (double)b) * (1.0 / 9007199254740992.0);
  }
};

// ---------------------------------------------------------------- CPython set
uint64_t tuple_hash(uint64_t x, uint64_t y) {
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P5 = 2870177450012600261ull;
  uint64_t acc = P5;
  for (uint64_t lane : {x, y}) {
    acc += lane * P2;
    acc = (acc << 31) | (acc >> 33);
    acc *= P1;
  }
  acc += 2ull ^ (P5 ^ 3527539ull);
  return acc == ~0ull ? 1546275796ull : acc;
}

constexpr int kNull = -1, kDummy = -2;
constexpr size_t kMinSize = 8, kLinearProbes = 9, kPerturbShift = 5;

struct PySet {
  std::vector<int32_t> key;   // cell id, kNull or kDummy
  std::vector<uint64_t> hash;
  size_t mask = kMinSize - 1, fill = 0, used = 0;

  PySet() : key(kMinSize, kNull), hash(kMinSize, 0) {}

  void insert_clean(int32_t k, uint64_t h) {  // set_insert_clean
    size_t perturb = h, i = h & mask;
    for (;;) {
      if (key[i] == kNull) break;
      bool found = false;
      if (i + kLinearProbes <= mask) {
        for (size_t j = 1; j <= kLinearProbes; ++j)
          if (key[i + j] == kNull) {
            i += j;
            found = true;
            break;
          }
      }
      if (found) break;
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
    }
    key[i] = k;
    hash[i] = h;
  }
  void resize(size_t minused) {  // set_table_resize
    size_t newsize = kMinSize;
    while (newsize <= minused) newsize <<= 1;
    std::vector<int32_t> ok;
    std::vector<uint64_t> oh;
    ok.swap(key);
    oh.swap(hash);
    key.assign(newsize, kNull);
    hash.assign(newsize, 0);
    mask = newsize - 1;
    fill = used;
    for (size_t j = 0; j < ok.size(); ++j)
      if (ok[j] >= 0) insert_clean(ok[j], oh[j]);
  }
  void add(int32_t k, uint64_t h) {  // set_add_entry (keys are distinct cells)
    size_t perturb = h, i = h & mask;
    long freeslot = -1;
    for (;;) {
      size_t probes = (i + kLinearProbes <= mask) ? kLinearProbes : 0;
      size_t e = i;
      for (;;) {
        if (key[e] == kNull) {
          if (freeslot >= 0) {
            ++used;
            key[freeslot] = k;
            hash[freeslot] = h;
            return;
          }
          ++fill;
          ++used;
          key[e] = k;
          hash[e] = h;
          if (fill * 5 < mask * 3) return;
          resize(used > 50000 ? used * 2 : used * 4);
          return;
        }
        if (key[e] == k) return;                    // already present
        if (key[e] == kDummy && freeslot < 0) freeslot = (long)e;
        if (probes == 0) break;
        --probes;
        ++e;
      }
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
    }
  }
  long find(int32_t k, uint64_t h) const {  // set_lookkey: slot of active k or -1
    size_t perturb = h, i = h & mask;
    for (;;) {
      size_t probes = (i + kLinearProbes <= mask) ? kLinearProbes : 0;
      size_t e = i;
      for (;;) {
        if (key[e] == kNull) return -1;
        if (key[e] == k) return (long)e;
        if (probes == 0) break;
        --probes;
        ++e;
      }
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
    }
  }
  void discard(int32_t k, uint64_t h) {  // set_discard_entry
    const long e = find(k, h);
    if (e < 0) return;
    key[e] = kDummy;
    hash[e] = ~0ull;  // -1
    --used;
  }
  // tail of set_difference_update_internal: more than 1/4 dummies -> resize away
  void settle_dummies() {
    if (fill - used > mask / 4) resize(used > 50000 ? used * 2 : used * 4);
  }
  // set_merge into THIS empty set (set_copy path of set_copy_and_difference)
  void merge_from(const PySet& o) {
    if ((fill + o.used) * 5 >= mask * 3) resize((used + o.used) * 2);
    if (fill == 0 && mask == o.mask && o.fill == o.used) {
      key = o.key;
      hash = o.hash;
      fill = o.fill;
      used = o.used;
      return;
    }
    fill = o.used;
    used = o.used;
    for (size_t j = 0; j <= o.mask; ++j)
      if (o.key[j] >= 0) insert_clean(o.key[j], o.hash[j]);
  }
  void list(std::vector<int32_t>& out) const {
    out.clear();
    for (size_t j = 0; j <= mask; ++j)
      if (key[j] >= 0) out.push_back(key[j]);
  }
};

}  // namespace

struct pe_pystream {
  int G, P, O;
  bool maze;         // map_generation_algo == 'maze' (the fork, plantos_env_new.py:355-358)
  double p_thirsty;
  Mt mt;
  PySet full;        // set((x, y) for x in range(G) for y in range(G)), fixed per G
  PySet full_copy;   // set_copy(full): the table set_copy_and_difference starts from
  std::vector<uint64_t> cell_hash;
  std::vector<int32_t> list, picks;
  std::vector<uint8_t> obst;
};

namespace {

// random.sample's set size threshold (random.py 3.10): 21 + 4 ** ceil(log(3k, 4))
int sample_setsize(int k) {
  int setsize = 21;
  if (k > 5) setsize += (int)std::pow(4.0, std::ceil(std::log((double)(k * 3)) / std::log(4.0)));
  return setsize;
}

// Obstacle clusters of _generate_map(_original), plantos_env.py:341-354; returns len(obstacles).
int clusters_original(pe_pystream* s) {
  const int G = s->G;
  Mt& mt = s->mt;
  std::fill(s->obst.begin(), s->obst.end(), 0);
  int n_obst = 0;
  for (int q = 0; q < s->O / 3; ++q) {                              // :341-343
    const int cx = 2 + (int)mt.below((uint32_t)(G - 4));            // randint(2, G-3)  :344
    const int cy = 2 + (int)mt.below((uint32_t)(G - 4));            // :345
    const int size = 2 + (int)mt.below(2u);                         // choice([2, 3])   :347
    for (int dx = 0; dx < size; ++dx)
      for (int dy = 0; dy < size; ++dy) {
        const int ox = cx + dx - size / 2, oy = cy + dy - size / 2; // :350-351
        if (0 <= ox && ox < G && 0 <= oy && oy < G && !s->obst[ox * G + oy]) {
          s->obst[ox * G + oy] = 1;                                 // obstacles.add   :353-354
          ++n_obst;
        }
      }
  }
  return n_obst;
}

// ---- the fork's maze, gradio-app/plantos_env_new.py:408-604 (obstacles only)
void carve(pe_pystream* s, int x, int y) {
  if (0 <= x && x < s->G && 0 <= y && y < s->G) s->obst[x * s->G + y] = 0;  // obstacles.discard
}

void maze_room(pe_pystream* s, int mx, int my) {                    // _carve_irregular_room :479-516
  Mt& mt = s->mt;
  const int bx = mx * 6 + 1, by = my * 6 + 1;
  for (int i = 0; i < 5; ++i)
    for (int j = 0; j < 5; ++j) carve(s, bx + i, by + j);
  if (mt.random() < 0.3)
    for (int i = 0; i < 2; ++i)
      for (int j = 2; j < 4; ++j) carve(s, bx + 5 + i, by + j);
  if (mt.random() < 0.3)
    for (int i = 2; i < 4; ++i)
      for (int j = 0; j < 2; ++j) carve(s, bx + i, by + 5 + j);
  if (mt.random() < 0.4) {
    static const int CORNER[4][2] = {{0, 0}, {4, 0}, {0, 4}, {4, 4}};
    const int k = (int)mt.below(4u);                                // random.choice(corners)
    const int x = bx + CORNER[k][0], y = by + CORNER[k][1];
    if (x < s->G && y < s->G) s->obst[x * s->G + y] = 1;             // obstacles.add
  }
}

void maze_path(pe_pystream* s, int cx, int cy, int nx, int ny) {    // :518-582
  if (cx == nx) {
    for (int m = std::min(cy, ny); m <= std::max(cy, ny); ++m)
      for (int i = 0; i < 5; ++i)
        for (int j = 0; j < 6; ++j) carve(s, cx * 6 + 1 + i, m * 6 + 1 + j);
  } else {
    for (int m = std::min(cx, nx); m <= std::max(cx, nx); ++m)
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 5; ++j) carve(s, m * 6 + 1 + i, cy * 6 + 1 + j);
  }
  if (s->mt.random() < 0.2) {                                       // _add_path_bulge
    const int mx = (cx + nx) / 2, my = (cy + ny) / 2;
    const int dir = s->mt.below(2u) ? 1 : -1;                       // random.choice([-1, 1])
    for (int i = 0; i < 2; ++i)
      for (int j = 0; j < 2; ++j) {
        if (cx == nx)
          carve(s, mx * 6 + 2 + dir * 2 + i, my * 6 + 2 + j);
        else
          carve(s, mx * 6 + 2 + i, my * 6 + 2 + dir * 2 + j);
      }
  }
}

// _generate_map_maze up to the plants (:408-456); returns len(obstacles).
int maze_obstacles(pe_pystream* s) {
  static const int DIRS[4][2] = {{0, 1}, {0, -1}, {1, 0}, {-1, 0}};
  const int G = s->G, mw = (G - 1) / 6;
  std::fill(s->obst.begin(), s->obst.end(), 1);
  std::vector<uint8_t> visited((size_t)mw * mw, 0);
  std::vector<int> stack;
  const int sx = (int)s->mt.below((uint32_t)mw), sy = (int)s->mt.below((uint32_t)mw);  // randint(0, meta-1)
  stack.push_back(sx * mw + sy);
  visited[sx * mw + sy] = 1;
  maze_room(s, sx, sy);
  while (!stack.empty()) {
    const int cx = stack.back() / mw, cy = stack.back() % mw;
    int cand[4], nc = 0;
    for (int d = 0; d < 4; ++d) {
      const int nx = cx + DIRS[d][0], ny = cy + DIRS[d][1];
      if (0 <= nx && nx < mw && 0 <= ny && ny < mw && !visited[nx * mw + ny]) cand[nc++] = d;
    }
    if (nc) {
      const int d = cand[s->mt.below((uint32_t)nc)];               // random.choice(neighbors)
      const int nx = cx + DIRS[d][0], ny = cy + DIRS[d][1];
      maze_path(s, cx, cy, nx, ny);
      maze_room(s, nx, ny);
      visited[nx * mw + ny] = 1;
      stack.push_back(nx * mw + ny);
    } else {
      stack.pop_back();
    }
  }
  int n = 0;
  for (uint8_t v : s->obst) n += v;
  return n;
}

// _generate_map for one env: cells u8[G*G] (pe_cell codes), rover (x, y).
int gen_one(pe_pystream* s, uint8_t* cells, int32_t* rover) {
  const int G = s->G, GG = G * G, P = s->P;
  Mt& mt = s->mt;
  int n_obst;
  if (s->maze) {
    n_obst = maze_obstacles(s);
    if (GG - n_obst < P + 1) n_obst = clusters_original(s);        // fallback, same stream (:461-466)
  } else {
    n_obst = clusters_original(s);
  }
  // available_positions = set(all) - obstacles   (:356-358, set_difference)
  PySet avail;
  if ((s->full.used >> 2) > (size_t)n_obst) {  // set_copy_and_difference
    avail = s->full_copy;
    for (int k = 0; k < GG; ++k)
      if (s->obst[k]) avail.discard(k, s->cell_hash[k]);
    avail.settle_dummies();
  } else {  // iterate so, add members not in other
    for (size_t j = 0; j <= s->full.mask; ++j) {
      const int32_t k = s->full.key[j];
      if (k >= 0 && !s->obst[k]) avail.add(k, s->full.hash[j]);
    }
  }
  if ((int)avail.used < P + 1) return PE_ERR_NOROOM;               // ValueError :360-364
  avail.list(s->list);
  const int n = (int)s->list.size();
  // plant_positions = random.sample(list(available_positions), P)   :366
  s->picks.resize(P);
  if (n <= sample_setsize(P)) {
    std::vector<int32_t> pool(s->list);
    for (int i = 0; i < P; ++i) {
      const int j = (int)mt.below((uint32_t)(n - i));
      s->picks[i] = pool[j];
      pool[j] = pool[n - i - 1];
    }
  } else {
    std::vector<uint8_t> selected(n, 0);
    for (int i = 0; i < P; ++i) {
      int j = (int)mt.below((uint32_t)n);
      while (selected[j]) j = (int)mt.below((uint32_t)n);
      selected[j] = 1;
      s->picks[i] = s->list[j];
    }
  }
  for (int k = 0; k < GG; ++k) cells[k] = s->obst[k] ? PE_OBSTACLE : PE_EMPTY;
  for (int i = 0; i < P; ++i)                                       // :367-369
    cells[s->picks[i]] = mt.random() < s->p_thirsty ? PE_THIRSTY : PE_HYDRATED;
  for (int i = 0; i < P; ++i) avail.discard(s->picks[i], s->cell_hash[s->picks[i]]);  // -= set(plants) :370
  avail.settle_dummies();
  avail.list(s->list);
  const int r = s->list[mt.below((uint32_t)s->list.size())];        // choice(list(...)) :372
  rover[0] = r / G;
  rover[1] = r % G;
  return PE_OK;
}

}  // namespace

extern "C" {

int pe_pystream_create(const pe_config* c, int64_t seed, pe_pystream** out) {
  if (!c || !out) return pe_internal_set_error(PE_ERR_ARG, "null argument");
  *out = nullptr;
  if (c->abi_version != PE_ABI_VERSION) return pe_internal_set_error(PE_ERR_ARG, "ABI version mismatch");
  const int G = c->grid_size;
  if (G < 5 && c->num_obstacles / 3 > 0)
    return pe_internal_set_error(PE_ERR_ARG, "randint(2, G-3) needs grid_size >= 5 (plantos_env.py:344)");
  if (G < 1 || G > 128 || c->num_plants < 0 || c->num_obstacles < 0)
    return pe_internal_set_error(PE_ERR_ARG, "bad geometry");
  if (c->map_generation_algo == PE_MAP_MAZE && G < 7)
    return pe_internal_set_error(PE_ERR_ARG, "the maze needs grid_size >= 7 (randint(0, (G-1)//6 - 1), "
                                             "plantos_env_new.py:427)");
  pe_pystream* s = new (std::nothrow) pe_pystream();
  if (!s) return pe_internal_set_error(PE_ERR_NOMEM, "host allocation failed");
  s->G = G;
  s->P = c->num_plants;
  s->O = c->num_obstacles;
  s->maze = c->map_generation_algo == PE_MAP_MAZE;
  s->p_thirsty = c->thirsty_plant_prob;
  s->mt.seed(seed < 0 ? (uint64_t)(-(seed + 1)) + 1u : (uint64_t)seed);  // random.seed: abs(a)
  s->cell_hash.resize((size_t)G * G);
  for (int x = 0; x < G; ++x)
    for (int y = 0; y < G; ++y) {
      s->cell_hash[x * G + y] = tuple_hash((uint64_t)x, (uint64_t)y);
      s->full.add(x * G + y, s->cell_hash[x * G + y]);  // set(generator): one add per item
    }
  s->full_copy.merge_from(s->full);
  s->obst.assign((size_t)G * G, 0);
  *out = s;
  return PE_OK;
}

int pe_pystream_next(pe_pystream* s, int32_t k, uint8_t* cells, int32_t* rover) {
  if (!s || k < 0 || (k > 0 && (!cells || !rover))) return pe_internal_set_error(PE_ERR_ARG, "null argument");
  const size_t GG = (size_t)s->G * s->G;
  for (int32_t j = 0; j < k; ++j) {
    const int rc = gen_one(s, cells + j * GG, rover + 2 * j);
    if (rc != PE_OK)
      return pe_internal_set_error(rc, "Not enough available positions to place the plants and the rover "
                                       "(plantos_env.py:360-364)");
  }
  return PE_OK;
}

uint32_t pe_pystream_getrandbits32(pe_pystream* s) { return s ? s->mt.next() : 0u; }

int pe_pystream_destroy(pe_pystream* s) {
  delete s;
  return PE_OK;
}

}  // extern "C"

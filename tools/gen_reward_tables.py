"""Derive the reward stack's data tables from the reference by PROBING its functions.

Run in the build container only (needs /root/reference):  python3 -B tools/gen_reward_tables.py
Writes (both generated from the same probe results, committed):
  pokegym_amd/reward_tables.py        plain-Python data for the oracle and host code
  pokegym_amd/csrc/pk_reward_tables.h C arrays for the K4 reward kernel

Nothing is parsed from source text: each table is what the imported reference functions return
when single RAM bits/bytes are set on a fake bus (tools/ref_env.py).
  MONITORS   ram_map_leanke.py monitor_{dojo,silph_co,hideout,poke_tower,gym3..7}_events:
             dict order, (addr, bit, weight) of every entry (environment.py:1457-1491 sums them
             with calculate_event_rewards, environment.py:1201-1219)
  DOJO_W     ram_map_leanke.py:793-814 dojo(): weight of each bit of D7B1
  BAG_NAMES  red_ram_api.py:404-422 Items._get_items_in_range names per item id -> the five
             names environment.py:1358-1372 looks for
  MAP_COORD  game_map.py:10-18 local_to_global offsets per map id (map_data.json)
  MAP_DIMS   constants.py MAP_DICT via MAP_ID_REF (environment.py:733-753 update_seen_map_dict)
  TREES      environment.py:60-80,277-312 tree grid positions in detect_and_reward_trees order
  MENU_*     red_memory_menus.py tables used by red_ram_api.py:149-225 get_battle_state
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import ref_env  # noqa: E402

MONITOR_NAMES = ["dojo", "silph_co", "hideout", "poke_tower", "gym3", "gym4", "gym5", "gym6", "gym7"]
BAG_TARGETS = ["Lemonade", "Silph Scope", "Lift Key", "Poke Doll", "Bicycle"]


class Bus:
    def __init__(self):
        self.mem = np.zeros(0x10000, np.uint8)

    def get_memory_value(self, a):
        return int(self.mem[a])

    def set_memory_value(self, a, v):
        self.mem[a] = v & 0xFF


def probe_monitor(fn):
    bus = Bus()
    keys = list(fn(bus).keys())
    found = {k: [] for k in keys}
    for addr in range(0xC000, 0xE000):
        bus.mem[addr] = 0xFF
        d = fn(bus)
        bus.mem[addr] = 0
        hit = [k for k in keys if d[k] != 0]
        if not hit:
            continue
        for bit in range(8):
            bus.mem[addr] = 1 << bit
            d = fn(bus)
            bus.mem[addr] = 0
            for k in keys:
                if d[k] != 0:
                    found[k].append((addr, bit, int(d[k])))
    out = []
    for k in keys:
        if len(found[k]) != 1:
            raise RuntimeError(f"monitor key {k}: expected one (addr, bit), got {found[k]}")
        out.append((k,) + found[k][0])
    return out


def main():
    E = ref_env.env_module()
    import pokegym.game_map as game_map
    import pokegym.ram_map_leanke as leanke
    import pokegym.constants as C
    import pokegym.bin.ram_reader.red_memory_items as items
    import pokegym.bin.ram_reader.red_memory_menus as menus

    monitors = {}
    for name in MONITOR_NAMES:
        monitors[name] = probe_monitor(getattr(leanke, f"monitor_{name}_events"))

    bus = Bus()
    dojo_w = []
    for bit in range(8):
        bus.mem[0xD7B1] = 1 << bit
        dojo_w.append(int(leanke.dojo(bus)))
    bus.mem[0xD7B1] = 0
    assert leanke.dojo(bus) == 0
    rng = np.random.default_rng(0)
    for v in rng.integers(0, 256, 64):
        bus.mem[0xD7B1] = v
        assert leanke.dojo(bus) == sum(w for b, w in enumerate(dojo_w) if v >> b & 1)

    # bag item names exactly as Items._get_items_in_range maps them
    def name_of(v):
        if v == 0xFF:
            return ""
        if v in items.ITEM_LOOKUP:
            return items.ITEM_LOOKUP[v]
        if v == 4:
            return "Pokeball"
        return ""
    bag_sets = {t: [v for v in range(256) if name_of(v) == t] for t in BAG_TARGETS}

    map_coord = {}
    for mid, e in game_map.MAP_DATA.items():
        if 0 <= mid <= 255:
            map_coord[mid] = tuple(int(x) for x in e["coordinates"])
    map_dims = {}
    for mid, name in C.MAP_ID_REF.items():
        d = C.MAP_DICT[name]
        map_dims[int(mid)] = (int(d["height"]), int(d["width"]))

    trees = []
    for y, x, m in E.TREE_POSITIONS_PIXELS:
        tx, ty = x // 16, y // 16
        cty = ty if not (tx == 212 and ty == 210) else 211
        trees.append((int(m), int(tx), int(cty)))

    MV, MK, SV = menus.RedRamMenuValues, menus.RedRamMenuKeys, menus.RedRamSubMenuValues
    menu_loc = sorted((int(k[0]), int(k[1]), int(v)) for k, v in menus.TEXT_MENU_CURSOR_LOCATIONS.items())
    item_loc = sorted((int(k), int(v)) for k, v in menus.TEXT_MENU_ITEM_LOCATIONS.items())
    menu_consts = {
        "MV_UNKNOWN": int(MV.UNKNOWN_MENU), "MV_PC_LOGOFF": int(MV.PC_LOGOFF), "MV_MENU_YES": int(MV.MENU_YES),
        "MV_MENU_NO": int(MV.MENU_NO), "MV_SELECT_STATS": int(MV.MENU_SELECT_STATS),
        "MV_SELECT_SWITCH": int(MV.MENU_SELECT_SWITCH), "MV_BATTLE_SWITCH": int(MV.BATTLE_SELECT_SWITCH),
        "MV_BATTLE_STATS": int(MV.BATTLE_SELECT_STATS), "MV_NAME_YES": int(MV.NAME_POKEMON_YES),
        "MV_NAME_NO": int(MV.NAME_POKEMON_NO), "MV_SWITCH_YES": int(MV.SWITCH_POKEMON_YES),
        "MV_SWITCH_NO": int(MV.SWITCH_POKEMON_NO), "MV_ITEM_QUANTITY": int(MV.ITEM_QUANTITY),
        "MV_ITEM_RANGE_ERROR": int(MV.ITEM_RANGE_ERROR), "SV_UNKNOWN": int(SV.UNKNOWN_MENU),
        "GS_UNKNOWN": int(E.Game.GameState.GAME_STATE_UNKNOWN), "GS_BATTLE_ANIMATION": int(E.Game.GameState.BATTLE_ANIMATION),
        "GS_BATTLE_TEXT": int(E.Game.GameState.BATTLE_TEXT),
    }
    item_keys = [MK.BATTLE_MART_PC_ITEM_1, MK.BATTLE_MART_PC_ITEM_2, MK.BATTLE_MART_PC_ITEM_N]
    menu_item_keys = [(int(a), int(b)) for a, b in item_keys]

    # ---- python data module
    py = ['"""Reward-stack data tables, GENERATED by tools/gen_reward_tables.py by probing the reference."""',
          "# ruff: noqa", ""]
    py.append("# (key, addr, bit, weight) in dict order, per ram_map_leanke monitor_*_events")
    py.append("MONITORS = {")
    for name, ents in monitors.items():
        py.append(f"    {name!r}: [")
        for k, a, b, w in ents:
            py.append(f"        ({k!r}, 0x{a:04X}, {b}, {w}),")
        py.append("    ],")
    py.append("}")
    py.append(f"DOJO_W = {dojo_w}  # weight of D7B1 bit 0..7 (ram_map_leanke.dojo)")
    py.append(f"BAG_TARGETS = {BAG_TARGETS!r}")
    py.append("BAG_IDS = {" + ", ".join(f"{t!r}: {v}" for t, v in bag_sets.items()) + "}")
    py.append("MAP_COORD = {" + ", ".join(f"{k}: {v}" for k, v in sorted(map_coord.items())) + "}  # id -> (x, y)")
    py.append("MAP_DIMS = {" + ", ".join(f"{k}: {v}" for k, v in sorted(map_dims.items())) + "}  # id -> (height, width)")
    py.append(f"TREES = {trees}  # (map, tree_x, tree_y) in TREE_POSITIONS_PIXELS order")
    py.append(f"MENU_LOC = {menu_loc}  # (cc30, cc31, RedRamMenuValues)")
    py.append(f"ITEM_LOC = {item_loc}")
    py.append(f"MENU_ITEM_KEYS = {menu_item_keys}")
    for k, v in menu_consts.items():
        py.append(f"{k} = {v}")
    open(os.path.join(REPO, "pokegym_amd", "reward_tables.py"), "w").write("\n".join(py) + "\n")

    # ---- C header
    h = ["// pk_reward_tables.h — GENERATED by tools/gen_reward_tables.py (probing the reference's",
         "// reward functions on a fake bus; see that script for the file:line of each table).",
         "#pragma once", "#include <stdint.h>", "",
         "// device-visible constant tables (the host-simulation build defines __constant__ away)",
         "#define PK_TBL __device__ __constant__", ""]
    allm = []
    starts = []
    for name in MONITOR_NAMES:
        starts.append(len(allm))
        allm += [(a, b, w) for _, a, b, w in monitors[name]]
    starts.append(len(allm))
    h.append(f"#define PK_NMON {len(MONITOR_NAMES)}")
    h.append(f"#define PK_NMON_ENT {len(allm)}")
    h.append("// monitors in order " + " ".join(MONITOR_NAMES) + "; entry = addr | bit<<16 | (weight+128)<<20")
    h.append("PK_TBL uint16_t pk_mon_start[PK_NMON + 1] = {" + ", ".join(map(str, starts)) + "};")
    h.append("PK_TBL uint32_t pk_mon_ent[PK_NMON_ENT] = {")
    for a, b, w in allm:
        h.append(f"    0x{a | (b << 16) | ((w + 128) << 20):08X}u,")
    h.append("};")
    h.append("PK_TBL int8_t pk_dojo_w[8] = {" + ", ".join(map(str, dojo_w)) + "};")
    bits = []
    for t in BAG_TARGETS:
        words = [0] * 8
        for v in bag_sets[t]:
            words[v >> 5] |= 1 << (v & 31)
        bits.append("{" + ", ".join(f"0x{w:08X}u" for w in words) + "}")
    h.append("// item-id bitmaps whose bag name is " + ", ".join(BAG_TARGETS))
    h.append("PK_TBL uint32_t pk_bag_name_bits[5][8] = {" + ", ".join(bits) + "};")
    mc = []
    for mid in range(256):
        if mid in map_coord:
            x, y = map_coord[mid]
            mc.append(f"{{{x}, {y}, 1}}")
        else:
            mc.append("{0, 0, 0}")
    h.append("// local_to_global offsets: {map_x, map_y, known}")
    h.append("PK_TBL int16_t pk_map_coord[256][3] = {" + ", ".join(mc) + "};")
    md = []
    for mid in range(256):
        if mid in map_dims:
            hh, ww = map_dims[mid]
            md.append(f"{{{hh}, {ww}, 1}}")
        else:
            md.append("{0, 0, 0}")
    h.append("// MAP_DICT dims via MAP_ID_REF: {height, width, known}")
    h.append("PK_TBL int16_t pk_map_dims[256][3] = {" + ", ".join(md) + "};")
    h.append(f"#define PK_NTREES {len(trees)}")
    h.append("PK_TBL int16_t pk_trees[PK_NTREES][3] = {" + ", ".join(f"{{{m}, {x}, {y}}}" for m, x, y in trees) + "};")
    h.append(f"#define PK_NMENU_LOC {len(menu_loc)}")
    h.append("PK_TBL uint32_t pk_menu_loc[PK_NMENU_LOC] = {" +
             ", ".join(f"0x{a | (b << 8) | (v << 16):06X}u" for a, b, v in menu_loc) + "};  // cc30 | cc31<<8 | value<<16")
    h.append(f"#define PK_NITEM_LOC {len(item_loc)}")
    h.append("PK_TBL uint16_t pk_item_loc[PK_NITEM_LOC][2] = {" + ", ".join(f"{{{k}, {v}}}" for k, v in item_loc) + "};")
    h.append("PK_TBL uint16_t pk_menu_item_keys[3] = {" + ", ".join(f"0x{a | (b << 8):04X}" for a, b in menu_item_keys) + "};")
    for k, v in menu_consts.items():
        h.append(f"#define PK_{k} {v}")
    open(os.path.join(REPO, "pokegym_amd", "csrc", "pk_reward_tables.h"), "w").write("\n".join(h) + "\n")
    print("monitors:", {k: len(v) for k, v in monitors.items()}, "dojo_w", dojo_w, "bag", bag_sets,
          "maps", len(map_coord), len(map_dims), "trees", len(trees), "menu_loc", len(menu_loc))


if __name__ == "__main__":
    main()

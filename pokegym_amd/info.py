"""The `info` telemetry record of Environment.step (environment.py:1621-1810), as K4 emits it.

On a step with `done or time % 10000 == 0` (:1621) the reward kernel writes one float64 record
per env (include/pokegym_amd.h `pk_info_ptr`, layout [PK_INFO_NFIELDS][npad]) and raises that
env's flag (`pk_info_flag_ptr`).  The record holds every numeric scalar of the reference's
info["stats"] and info["reward"] dicts, in the order below (`levels` as its six raw entries).

For an empty party the reference's "highest_pokemon_level" (max(party_levels), :1672) raises
ValueError while it builds the dict; the device then records PK_ERR_EMPTY_PARTY for the env (no
record), and Environment / VecEnv raise ValueError as the reference does.

"coord" (np.sum of the 444x436 counts_map heat map, :648-679) is in the record when the heat map
is kept (PK_F_HEATMAP; NaN otherwise); the map itself ("pokemon_exploration_map") is a device
array (pk_heatmap_ptr).  Not in the record: "maps_explored" (np.sum over a Python set — not a
number in the reference).  The detailed_rewards_* / *_events_aggregate dicts come from the 130
event-monitor bits K4 stores beside the record (pk_info_bits_ptr, event_dicts below).
"""
from __future__ import annotations

STATS_FIELDS = (
    "step", "x", "y", "map", "pcount",
    "levels_0", "levels_1", "levels_2", "levels_3", "levels_4", "levels_5",
    "levels_sum", "deaths", "deaths_per_episode", "badges", "self.badge_count",
    "badge_1", "badge_2", "badge_3", "badge_4", "badge_5", "badge_6",
    "events", "opponent_level",
    "met_bill", "used_cell_separator_on_bill", "ss_ticket", "met_bill_2",
    "bill_said_use_cell_separator", "left_bills_house_after_helping", "got_hm01", "rubbed_captains_back",
    "party_size", "highest_pokemon_level", "total_party_level", "event", "money",
    "seen_npcs_count", "seen_pokemon", "caught_pokemon", "moves_obtained", "hidden_obj_count",
    "bill_saved", "hm_count", "cut_taught", "bill_capt", "cut_coords", "cut_tiles",
    "bag_menu", "stats_menu", "pokemon_menu", "start_menu", "used_cut",
    "state_loaded_instead_of_resetting_in_game", "defeated_fighting_dojo", "got_hitmonlee", "got_hitmonchan",
    "coord",   # np.sum(counts_map): needs the heat map (PK_F_HEATMAP); NaN in the record without it
)

REWARD_FIELDS = (
    "delta", "event", "level", "opponent_level", "death", "badges", "bill_saved_reward", "hm_count_reward",
    "healing", "exploration", "seen_pokemon_reward", "caught_pokemon_reward", "moves_obtained_reward",
    "used_cut_reward", "tree_distance_reward", "dojo_reward_old",
    "has_lemonade_in_bag_reward", "has_silph_scope_in_bag_reward", "has_lift_key_in_bag_reward",
    "has_pokedoll_in_bag_reward", "has_bicycle_in_bag_reward",
)

FIELDS = STATS_FIELDS + tuple("reward." + k for k in REWARD_FIELDS)
NFIELDS = len(FIELDS)           # == PK_INFO_NFIELDS (include/pokegym_amd.h)

# stats entries the reference stores as Python floats (float(...), /5, * 0.1 ...); the rest are ints
_FLOAT_STATS = frozenset(("badges", "badge_1", "badge_2", "badge_3", "badge_4", "badge_5", "badge_6",
                          "bill_capt", "cut_coords", "cut_tiles", "bag_menu", "stats_menu", "pokemon_menu",
                          "start_menu"))


def reference_value(stats: dict, key: str):
    """The reference info["stats"] entry a STATS_FIELDS key names (tools/make_golden_info.py)."""
    if key[:7] == "levels_" and key[7:].isdigit():
        return stats["levels"][int(key[7:])]
    return stats[key]


def info_dict(values) -> dict:
    """One env's record (NFIELDS float64 values) -> {"stats": {...}, "reward": {...}} with the
    reference's keys and Python number types."""
    ns = len(STATS_FIELDS)
    stats = {}
    for k, v in zip(STATS_FIELDS, values[:ns]):
        if k[:7] == "levels_" and k[7:].isdigit():
            continue
        if k == "coord":
            if v == v:   # not NaN: the heat map is kept
                stats[k] = float(v)
            continue
        stats[k] = float(v) if k in _FLOAT_STATS else int(v)
    stats["levels"] = [int(v) for v in values[5:11]]
    reward = {k: float(v) for k, v in zip(REWARD_FIELDS, values[ns:])}
    return {"stats": stats, "reward": reward}


# ---- event-monitor dicts (environment.py:1706-1808): K4 emits the 130 monitor bits ----------
def _monitors():
    from . import reward_tables as T
    return T.MONITORS


def event_values(bits) -> list:
    """Monitor bits (u32 words, reward_tables.MONITORS order) -> weight * bit per entry."""
    out, i = [], 0
    for ents in _monitors().values():
        for _, _, _, wgt in ents:
            out.append(wgt * ((int(bits[i >> 5]) >> (i & 31)) & 1))
            i += 1
    return out


def detailed(v: int, base: int = 10, inc: int = 2, mult: int = 1):
    """calculate_event_rewards_detailed (environment.py:1221-1231) for one event value."""
    return base + v * inc * mult if v > 0 else v * inc * mult


def event_dicts(bits) -> dict:
    """The reference info dict's detailed_rewards_* and *_events_aggregate entries."""
    vals = iter(event_values(bits))
    agg = {k: {name: next(vals) for name, _, _, _ in ents} for k, ents in _monitors().items()}
    det = {k: {n: detailed(v) for n, v in d.items()} for k, d in agg.items()}
    return {
        "detailed_rewards_silph_co": det["silph_co"], "detailed_rewards_dojo": det["dojo"],
        "detailed_rewards_hideout": det["hideout"], "detailed_rewards_poke_tower": det["poke_tower"],
        "detailed_rewards_gyms": {f"gym_{g}_detailed_rewards": det[f"gym{g}"] for g in range(3, 8)},
        "silph_co_events_aggregate": agg["silph_co"], "dojo_events_aggregate": agg["dojo"],
        "hideout_events_aggregate": agg["hideout"], "poke_tower_events_aggregate": agg["poke_tower"],
        "gym_events": {f"gym_{g}_events": agg[f"gym{g}"] for g in range(3, 8)},
    }

from .network import (LAYOUT, PARAM_SHAPES, ArenaLayout, Network, arena_state_dict,
                      init_arena, load_state_dict_into, network_from_arena)

__all__ = ["LAYOUT", "PARAM_SHAPES", "ArenaLayout", "Network", "arena_state_dict",
           "init_arena", "load_state_dict_into", "network_from_arena"]

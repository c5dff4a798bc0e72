// ggrs_amd/csrc/plugin.hip — a user's game compiled against the engine's
// kernels into a plugin library (include/ggrs_amd_game.hpp contract).
//
//   hipcc <engine flags> -shared -include <game header> -DRB_PLUGIN_GAME=<struct> \
//         -o libggrs_game_<name>.so ggrs_amd/csrc/plugin.hip
// (make -C ggrs_amd/csrc plugin GAME_HEADER=... GAME=... PLUGIN_OUT=..., or
// ggrs_amd.plugin.build_game_plugin).  rb_register_game_plugin (engine.hip)
// dlopens the library and creates the game's GameOps through
// rb_plugin_make_ops: every kernel of the engine (SyncTest ticks, fused steady
// ticks, P2P ticks, checksum reports) is instantiated here for the game, so
// the plugin's own code object carries them.
#include "../../include/ggrs_amd_game.hpp"
#include "kernels.hpp"

#ifndef RB_PLUGIN_GAME
#error "compile with -include <game header> -DRB_PLUGIN_GAME=<game struct>"
#endif

extern "C" {

int32_t rb_plugin_abi() { return RB_PLUGIN_ABI; }

int32_t rb_plugin_players() { return RB_PLUGIN_GAME::kPlayers; }

// A new GameOps for `players` (must be the game's kPlayers), owned by the caller
// (deleted through its virtual destructor); NULL on a mismatch.
rb::GameOps* rb_plugin_make_ops(int32_t players, int32_t abi) {
  if (abi != RB_PLUGIN_ABI || players != RB_PLUGIN_GAME::kPlayers) return nullptr;
  return new rb::GameOpsT<rb::PluginGame<RB_PLUGIN_GAME>>();
}

}  // extern "C"

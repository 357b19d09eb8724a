"""Toot-and-Otto board sizes.  The device key holds every
board of at most 24 cells (two A-bit planes + 16 hand bits); a board of more cells cannot be
played to the end under the reference's rules -- each player has 6 T and 6 O whatever the
board -- because the 24 pieces can run out on a board that is not full with TOOT and OTTO
tied: a position with no move that is not primitive, where the reference's solver hangs
(SURVEY Appendix A).  tools/toot_stuck_positions.py finds such positions."""
import os
import sys

import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))
import toot_stuck_positions as tsp  # noqa: E402


@pytest.mark.parametrize("L,H", [(5, 5), (7, 4)])
def test_boards_above_24_cells_reach_a_position_without_moves(L, H):
    t, b = tsp.find_stuck(L, H)
    assert len(b) == 24 < L * H
    sc = tsp.words(b, L, H)
    assert sc["TOOT"] == sc["OTTO"]
    # gravity: every column is filled from the bottom without gaps
    for x in range(L):
        ys = sorted(y for (xx, y) in b if xx == x)
        assert ys == list(range(len(ys)))


@pytest.mark.parametrize("L,H", [(6, 4), (4, 6), (8, 3), (3, 8), (5, 4)])
def test_boards_of_at_most_24_cells_fill_before_the_hands_run_out(L, H):
    assert L * H <= 24      # 24 pieces >= cells: no move only on a full board (primitive)
    assert tsp.find_stuck(L, H, tries=50) is None


def test_descriptor_takes_every_board_of_at_most_24_cells():
    from gamesmanmpi_amd import Context, GMError, _lib
    for L, H in [(6, 4), (4, 6), (8, 3), (3, 8), (5, 4), (7, 3)]:
        Context(_lib.GAME_TOOT, (L, H)).close()
    for L, H in [(5, 5), (7, 4)]:
        with pytest.raises(GMError):
            Context(_lib.GAME_TOOT, (L, H))

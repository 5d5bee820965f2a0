"""Host-side helpers of the round-6 glue paths (CPU): the row-stride test that decides whether a
gradient slice is read in place (attention._rows_ld), and the positional-gradient mailbox hand-over
(attention._take_gx) -- no kernel runs here."""
import torch

from svdformer_pointsea_amd import attention as A


def test_rows_ld_contiguous_and_channel_slices():
    t = torch.zeros(2, 300, 1024)
    assert A._rows_ld(t) == 1024
    half = t[..., 512:]                  # the concatenation's second half: rows 1024 apart
    assert A._rows_ld(half) == 1024
    assert A._rows_ld(t[..., :512]) == 1024
    assert A._rows_ld(t.reshape(600, 1024)[:, 256:512]) == 1024


def test_rows_ld_rejects_uneven_and_transposed():
    t = torch.zeros(2, 300, 1024)
    assert A._rows_ld(t[:, :150, :512]) is None         # half the rows of each batch: batch stride != rows x ld
    assert A._rows_ld(t[:, ::2, :512]) == 2048           # every other row: still evenly spaced (150 x 2048)
    assert A._rows_ld(t.transpose(1, 2)) is None         # column stride != 1
    assert A._rows_ld(t[..., 1:513]) is None             # 4-byte offset: not 16-byte aligned
    assert A._rows_ld(torch.zeros(4, 12)[:, :6]) is None  # ld 12 is not a multiple of 8
    # a single-row batch dimension does not constrain its stride
    assert A._rows_ld(torch.zeros(1, 5, 64)[..., :32]) == 64


def test_take_gx_is_taken_once():
    class Ctx:
        pass

    ctx = Ctx()
    assert A._take_gx(ctx) is None                      # no mailbox
    ctx.gx_box = []
    assert A._take_gx(ctx) is None                      # empty mailbox

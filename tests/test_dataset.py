"""Host-side input pipeline (CPU): sample construction and padding of the reference's dataset schema
(src/custom_dataset.py:9-132), restated in ergm_amd.dataset."""
import torch

from ergm_amd.dataset import DialogueDataset, PadCollate

SP1, SP2, EOS = 98, 99, 97


def _schema():
    # two dialogues; dialogue 0 has two utterances, dialogue 1 one (too long -> skipped) + one short
    txt = [
        [[[1, 2, 3], [4, 5]], [[6, 7], [8], [9, 10, 11]]],
        [[list(range(20))] * 60, [[12, 13]]],
    ]
    label = [
        [[50, 51, 30, 31, 60, 61], [50, 51, 40, 41, 42, 43, 44, 45, 46, 47, 60, 61]],
        [[50, 51, 1, 60, 61], [50, 51, 2, 60, 61]],
    ]
    img = [[torch.full((8,), 0.5)], [torch.full((8,), -1.0)]]
    aud = [[torch.full((8,), 2.0)], [torch.full((8,), 3.0)]]
    context = [[[70, 71], [72]], [[73], [74, 75, 76]]]
    emo = [[3, 4], [5, 6]]
    return {"txt": txt, "img": img, "aud": aud, "label": label}, {"context": context, "label": emo}


def test_sample_construction_follows_reference_rules():
    data, ctx = _schema()
    ds = DialogueDataset(data, ctx, sp1_id=SP1, sp2_id=SP2, eos_id=EOS)
    assert len(ds) == 3  # the 1200-token utterance is dropped (>= 1024, src/custom_dataset.py:50-51)
    ids, tt, lm, vis, aud, c, e = ds[0]
    assert ids == [1, 2, 3, 4, 5]
    assert tt == [SP1, SP1, SP1, SP2, SP2]
    assert lm == [-100, -100, 30, 31, EOS]          # target[2:-2] + eos, right-aligned
    assert torch.equal(vis, torch.full((8,), 0.5)) and torch.equal(aud, torch.full((8,), 2.0))
    assert c == [70, 71] and e == 3
    ids, tt, lm, *_ = ds[1]                          # target longer than the input: input eos-padded
    assert lm == [40, 41, 42, 43, 44, 45, 46, 47, EOS]
    assert ids == [6, 7, 8, 9, 10, 11, EOS, EOS, EOS]
    assert tt == [SP1, SP1, SP2, SP1, SP1, SP1, SP1, SP1, SP1]
    assert ds[2][6] == 6


def test_pad_collate():
    data, ctx = _schema()
    ds = DialogueDataset(data, ctx, sp1_id=SP1, sp2_id=SP2, eos_id=EOS)
    b = PadCollate(eos_id=EOS, pad_multiple=4)([ds[0], ds[1], ds[2]])
    assert b["input_ids"].shape == (3, 12)           # longest 9, rounded up to a multiple of 4
    assert b["input_ids"][0, 5:].eq(EOS).all() and b["token_type_ids"][0, 5:].eq(EOS).all()
    assert b["labels"][0, 5:].eq(-100).all() and b["labels"][1, 8] == EOS
    assert b["caption_ids"][2, :3].tolist() == [74, 75, 76] and b["caption_ids"][2, 3:].eq(EOS).all()
    assert b["visual_feat"].shape == (3, 8) and b["audio_feat"][2, 0] == 3.0
    assert b["emotion_labels"].tolist() == [3, 4, 6]

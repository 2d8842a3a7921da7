"""Native WordPiece tokenizer: both vocab conventions, batching, truncation."""
from libsplinter_amd.models.tokenizer import WordPieceTokenizer, synthetic_vocab

BERT = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "hello", "world", "##s", "un", "##aff", "##able", ",", "!", "cafe"]


def test_bert_hash_convention():
    t = WordPieceTokenizer(BERT)
    assert not t.wpm
    assert t.encode("Hello worlds, unaffable!") == [2, 4, 5, 6, 10, 7, 8, 9, 11, 3]
    assert t.encode("xyz") == [2, 1, 3]
    assert t.encode("CAFÉ") == [2, 12, 3]  # lowercase + accent strip
    assert t.encode("", add_special=False) == []


def test_gguf_wpm_convention_and_decode():
    v = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "▁hello", "▁world", "s", "▁un", "aff", "able", "▁,"]
    t = WordPieceTokenizer(v)
    assert t.wpm
    assert t.encode("hello worlds un affable") == [2, 4, 5, 6, 7, 1, 3]
    ids = t.encode("hello world")
    assert t.decode(ids) == "hello world"


def test_batch_and_truncation():
    t = WordPieceTokenizer(synthetic_vocab())
    texts = ["the search", "a " * 50, "x"]
    ids, offs, full = t.encode_batch(texts, 16)
    assert list(full) == [len(t.encode(x)) for x in texts]
    assert offs[1] - offs[0] == full[0]
    assert offs[2] - offs[1] == 16 and ids[offs[2] - 1] == t.sep_id  # truncated, [SEP] kept
    assert ids[0] == t.cls_id


def test_unicode_and_punct_split():
    t = WordPieceTokenizer(synthetic_vocab())
    a = t.encode("vector,store!")
    b = t.encode("vector , store !")
    assert a == b
    assert t.encode("中文") == [t.cls_id, t.unk_id, t.unk_id, t.sep_id]

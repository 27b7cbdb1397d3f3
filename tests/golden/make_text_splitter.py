#!/usr/bin/env python3
"""Generate tests/golden/text_splitter.json: inputs and the reference's own
TextSplitter outputs (src/genie_tts/Utils/TextSplitter.py, pure Python, loaded by
path in the build container only).  Data only: input strings and split lists."""
import json
import os
import runpy

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/src/genie_tts/Utils/TextSplitter.py"

CASES = [
    "",
    "こんにちは。",
    "今日はいい天気ですね。散歩に行きましょう！",
    "短い。はい。そうですか、わかりました。",
    "Hello world. This is a test! Is it working? Yes.",
    "Hi. Ok. Fine, thanks.",
    "这是一个很长的句子，没有结束符号，但是有很多逗号，逗号，逗号，逗号，逗号，逗号，逗号，逗号，继续写下去",
    "他说：“你好！”然后离开了……真的吗？！",
    "第一行\n第二行。第三行",
    "ああ......そうか。",
    "——破折号——测试。结束",
    "末尾の句読点だけ。。。",
    "A, b, c, d, e, f, g, h, i, j, k, l, m, n, o, p, q, r, s, t, u, v, w, x, y, z, and more words here.",
    "混合English和中文的句子。Another sentence here! 最后",
    "...",
    "。。。あ",
    "ねえ、ちょっと待って；今行くから：すぐに。",
    "'quoted' and \"double\" marks; semicolons: colons.",
]


def main():
    ts = runpy.run_path(REF)["TextSplitter"]
    out = []
    for text in CASES:
        for max_len, min_len in ((40, 5), (20, 3)):
            out.append({"text": text, "max_len": max_len, "min_len": min_len,
                        "split": ts(max_len=max_len, min_len=min_len).split(text)})
    with open(os.path.join(HERE, "text_splitter.json"), "w", encoding="utf-8") as f:
        json.dump(out, f, ensure_ascii=False, indent=1)
    print(len(out), "cases")


if __name__ == "__main__":
    main()

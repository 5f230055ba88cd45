"""Reference error chains (transfer.go:192-196, issue/verifier.go:40-56,
rangecorrectness.go:141-160) -> (fts_status, fail index): test helper."""
RP_STATUS = {"invalid range proof": 3, "invalid IPA": 6, "invalid range proof: nil elements": 2,
             "invalid IPA proof: nil elements": 4, "invalid IPA proof": 5}


def classify(err, idx=-1):
    if err is None:
        return (0, -1)
    for prefix in ("invalid transfer proof: ", "invalid issue proof: "):
        if err.startswith(prefix):
            err = err[len(prefix):]
    if err == "invalid sum and type proof":
        return (8, -1)
    if err == "invalid same type proof":
        return (9, -1)
    if err == "invalid range proof":
        return (7, -1)
    if err.startswith("invalid range proof at index"):
        return (RP_STATUS[err.split(": ", 1)[1]], idx)
    return (1, -1)

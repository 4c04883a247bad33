"""Literal restatement of the reference's SLO-prediction harness
(ML/HTM/ModelTesting.py:36-171) for one stream.  TEST INFRASTRUCTURE ONLY:
the checker for the batched harness and for the statistical comparison with
ML/Data/result_model1.txt.
"""

MAX_LEAD_TIME = 50          # ModelTesting.py:31
SLO_RESPONSE_TIME = 70      # ModelTesting.py:32


def evaluate(windows, means, violations, threshold, max_lead=MAX_LEAD_TIME, cut=None, labels=None):
    """windows[r] = the 1+7 anomaly scores of record r (ModelTesting.py:66-72).
    Returns (tp, fp, tn, fn, avg_lead or None) as getModelStats prints them.
    For oracle/label_rule_search.py only: `cut` (default max_lead) is the tail
    getModelStats leaves out, `labels` (0/1 per record) replaces :57-60's rule."""
    cut = max_lead if cut is None else cut
    pl = []
    for r0, win in enumerate(windows):
        rcount = r0 + 1                                        # :62
        if labels is not None:
            violation = int(labels[r0])
        else:
            violation = 1 if (violations[r0] > 0 or means[r0] >= SLO_RESPONSE_TIME) else 0   # :57-60
        n_over = sum(1 for a in win if float(a) > threshold)   # :75-77 (float32 vs double)
        if n_over > 0 and rcount > 1:                          # :81
            pl.append([-1, 'A', rcount, 'TP', 0])
        else:
            pl.append([-1, 'N', rcount, 'TN'])
        state = 'A' if violation > 0 else 'N'                  # :101-107
        for item in pl:                                        # processpredictionList :113-146
            if item[0] != -1:
                continue
            if state == 'A':
                if item[1] == 'N':
                    if rcount - item[2] <= max_lead:
                        item[3] = 'FN'
                        item[0] = 0
                else:
                    if rcount - item[2] <= max_lead:
                        item[3] = 'TP'
                        item[0] = 0
                        item[4] = max_lead - (rcount - item[2])
                        start = rcount - max_lead if rcount - max_lead > 0 else 0
                        for nelem in pl[start:rcount]:
                            if nelem[3] == 'FN':
                                nelem[3] = 'TN'
            else:
                if item[1] == 'A':
                    if rcount - item[2] > max_lead:
                        item[3] = 'FP'
                        item[0] = 0
                else:
                    if rcount - item[2] > max_lead:
                        item[3] = 'TN'
                        item[0] = 0
    tp = fp = tn = fn = 0
    lead = 0.0
    for item in pl[:-cut]:                                     # getModelStats :148-171
        if item[3] == 'TP':
            tp += 1
            lead += item[4]
        elif item[3] == 'TN':
            tn += 1
        elif item[3] == 'FP':
            fp += 1
        elif item[3] == 'FN':
            fn += 1
    return tp, fp, tn, fn, (lead / tp if tp else None)

// gosort.h — TEST INFRASTRUCTURE (oracle). Restatement of Go's sort.Slice
// (src/sort/zsortfunc.go, pattern-defeating quicksort, Go >= 1.19), needed
// because karpenter-core re-sorts in-flight NodeClaims with the unstable
// sort.Slice for every pod (<U> scheduler.go add()), so tie order decides
// which NodeClaim a pod lands on.
#pragma once
#include <cstdint>

namespace gosort {

inline int bits_len(uint64_t x) {
  int n = 0;
  while (x) { ++n; x >>= 1; }
  return n;
}

struct XorShift {
  uint64_t s;
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
};

enum Hint { kUnknown = 0, kIncreasing = 1, kDecreasing = 2 };

template <class D>
struct Sorter {
  D& d;  // d.less(i,j), d.swap(i,j)

  void insertion_sort(int a, int b) {
    for (int i = a + 1; i < b; i++)
      for (int j = i; j > a && d.less(j, j - 1); j--) d.swap(j, j - 1);
  }
  void sift_down(int lo, int hi, int first) {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && d.less(first + child, first + child + 1)) child++;
      if (!d.less(first + root, first + child)) return;
      d.swap(first + root, first + child);
      root = child;
    }
  }
  void heap_sort(int a, int b) {
    int first = a, lo = 0, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; i--) sift_down(i, hi, first);
    for (int i = hi - 1; i >= 0; i--) {
      d.swap(first, first + i);
      sift_down(lo, i, first);
    }
  }
  void pdqsort(int a, int b, int limit) {
    const int maxInsertion = 12;
    bool wasBalanced = true, wasPartitioned = true;
    for (;;) {
      int length = b - a;
      if (length <= maxInsertion) {
        insertion_sort(a, b);
        return;
      }
      if (limit == 0) {
        heap_sort(a, b);
        return;
      }
      if (!wasBalanced) {
        break_patterns(a, b);
        limit--;
      }
      int hint;
      int pivot = choose_pivot(a, b, &hint);
      if (hint == kDecreasing) {
        reverse_range(a, b);
        pivot = (b - 1) - (pivot - a);
        hint = kIncreasing;
      }
      if (wasBalanced && wasPartitioned && hint == kIncreasing) {
        if (partial_insertion_sort(a, b)) return;
      }
      if (a > 0 && !d.less(a - 1, pivot)) {
        int mid = partition_equal(a, b, pivot);
        a = mid;
        continue;
      }
      bool alreadyPartitioned;
      int mid = partition(a, b, pivot, &alreadyPartitioned);
      wasPartitioned = alreadyPartitioned;
      int leftLen = mid - a, rightLen = b - mid;
      int balanceThreshold = length / 8;
      if (leftLen < rightLen) {
        wasBalanced = leftLen >= balanceThreshold;
        pdqsort(a, mid, limit);
        a = mid + 1;
      } else {
        wasBalanced = rightLen >= balanceThreshold;
        pdqsort(mid + 1, b, limit);
        b = mid;
      }
    }
  }
  int partition(int a, int b, int pivot, bool* already) {
    d.swap(a, pivot);
    int i = a + 1, j = b - 1;
    while (i <= j && d.less(i, a)) i++;
    while (i <= j && !d.less(j, a)) j--;
    if (i > j) {
      d.swap(j, a);
      *already = true;
      return j;
    }
    d.swap(i, j);
    i++;
    j--;
    for (;;) {
      while (i <= j && d.less(i, a)) i++;
      while (i <= j && !d.less(j, a)) j--;
      if (i > j) break;
      d.swap(i, j);
      i++;
      j--;
    }
    d.swap(j, a);
    *already = false;
    return j;
  }
  int partition_equal(int a, int b, int pivot) {
    d.swap(a, pivot);
    int i = a + 1, j = b - 1;
    for (;;) {
      while (i <= j && !d.less(a, i)) i++;
      while (i <= j && d.less(a, j)) j--;
      if (i > j) break;
      d.swap(i, j);
      i++;
      j--;
    }
    return i;
  }
  bool partial_insertion_sort(int a, int b) {
    const int maxSteps = 5, shortestShifting = 50;
    int i = a + 1;
    for (int j = 0; j < maxSteps; j++) {
      while (i < b && !d.less(i, i - 1)) i++;
      if (i == b) return true;
      if (b - a < shortestShifting) return false;
      d.swap(i, i - 1);
      if (i - a >= 2) {
        for (int k = i - 1; k >= 1; k--) {
          if (!d.less(k, k - 1)) break;
          d.swap(k, k - 1);
        }
      }
      if (b - i >= 2) {
        for (int k = i + 1; k < b; k++) {
          if (!d.less(k, k - 1)) break;
          d.swap(k, k - 1);
        }
      }
    }
    return false;
  }
  void break_patterns(int a, int b) {
    int length = b - a;
    if (length >= 8) {
      XorShift r{(uint64_t)length};
      uint64_t modulus = 1ull << bits_len((uint64_t)length);
      int idx = a + (length / 4) * 2 - 1;
      for (int i = 0; i < 3; i++) {
        int other = (int)((uint64_t)r.next() & (modulus - 1));
        if (other >= length) other -= length;
        d.swap(idx - 1 + i, a + other);
      }
    }
  }
  int choose_pivot(int a, int b, int* hint) {
    const int shortestNinther = 50, maxSwaps = 4 * 3;
    int l = b - a;
    int swaps = 0;
    int i = a + l / 4 * 1, j = a + l / 4 * 2, k = a + l / 4 * 3;
    if (l >= 8) {
      if (l >= shortestNinther) {
        i = median_adjacent(i, &swaps);
        j = median_adjacent(j, &swaps);
        k = median_adjacent(k, &swaps);
      }
      j = median(i, j, k, &swaps);
    }
    if (swaps == 0) *hint = kIncreasing;
    else if (swaps == maxSwaps) *hint = kDecreasing;
    else *hint = kUnknown;
    return j;
  }
  void order2(int& a, int& b, int* swaps) {
    if (d.less(b, a)) {
      (*swaps)++;
      int t = a;
      a = b;
      b = t;
    }
  }
  int median(int a, int b, int c, int* swaps) {
    order2(a, b, swaps);
    order2(b, c, swaps);
    order2(a, b, swaps);
    return b;
  }
  int median_adjacent(int a, int* swaps) { return median(a - 1, a, a + 1, swaps); }
  void reverse_range(int a, int b) {
    int i = a, j = b - 1;
    while (i < j) {
      d.swap(i, j);
      i++;
      j--;
    }
  }
};

// sort.Slice(x, less): limit = bits.Len(uint(length))
template <class D>
void slice(D& d, int n) {
  Sorter<D> s{d};
  s.pdqsort(0, n, bits_len((uint64_t)n));
}

}  // namespace gosort

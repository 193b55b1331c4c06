// concepts.hh — the functor contracts of the operator surface (reference: concepts.hh:23-86).
// Same concept names and requirements, so the drivers' functors are checked as before.
#pragma once

#include <concepts>
#include <ostream>

#if __cplusplus < 202002L
#error "the hj3d drop-in headers need C++20 (concepts)"
#endif

template <typename T>
concept Printable = requires(std::ostream& os, T a) { os << a; };

// static output_t eval(const input_t*)
template <typename T>
concept alg_hashfun_c = requires {
  typename T::input_t;
  typename T::output_t;
  { T::eval(static_cast<const typename T::input_t*>(nullptr)) } -> std::same_as<typename T::output_t>;
};

// static bool eval(const input_t*)
template <typename T>
concept alg_predicate_c = requires {
  typename T::input_t;
  { T::eval(static_cast<const typename T::input_t*>(nullptr)) } -> std::same_as<bool>;
};

// bool operator()(const input_t*)
template <typename T>
concept alg_dyn_predicate_c = requires(T t) {
  typename T::input_t;
  { t(static_cast<const typename T::input_t*>(nullptr)) } -> std::same_as<bool>;
};

// static bool eval(const left_t*, const right_t*)
template <typename T>
concept alg_binary_predicate_c = requires {
  typename T::left_t;
  typename T::right_t;
  { T::eval(static_cast<const typename T::left_t*>(nullptr), static_cast<const typename T::right_t*>(nullptr)) }
      -> std::same_as<bool>;
};

// static output_t eval(left_t*, right_t*)
template <typename T>
concept alg_concatfun_c = requires {
  typename T::left_t;
  typename T::right_t;
  typename T::output_t;
  { T::eval(static_cast<typename T::left_t*>(nullptr), static_cast<typename T::right_t*>(nullptr)) }
      -> std::same_as<typename T::output_t>;
};

// eval_left / eval_right / getMainNode over a nested tuple
template <typename T>
concept alg_unnestfun_c = requires {
  typename T::input_t;
  typename T::output_t;
  typename T::MainNode;
  typename T::data_t;
  { T::eval_left(static_cast<typename T::output_t*>(nullptr), static_cast<typename T::input_t*>(nullptr)) }
      -> std::same_as<void>;
  { T::eval_right(static_cast<typename T::output_t*>(nullptr), static_cast<typename T::input_t*>(nullptr),
                  static_cast<const typename T::data_t*>(nullptr)) } -> std::same_as<void>;
  { T::getMainNode(static_cast<typename T::input_t*>(nullptr)) } -> std::same_as<const typename T::MainNode*>;
};

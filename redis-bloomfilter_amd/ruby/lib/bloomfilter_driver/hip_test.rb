# frozen_string_literal: true

# Redis::BloomfilterDriver::HipTest — lib/bloomfilter_driver/ruby_test.rb's hash engines
# on the device (`driver: 'hip-test'`, resolved by const_get like every driver).
#
# Probe i of a key is Digest::<E>.hexdigest("#{i}-#{key}").to_i(16) % bits
# (ruby_test.rb:43-61), E = options[:hash_engine] ('md5' by default, bloomfilter.rb:15):
# the filter is created with BF_FLAG_ENGINE_MD5 / BF_FLAG_ENGINE_SHA1 and everything
# else is the Hip driver's.  'crc32' is broken upstream (Integer#to_i takes no radix,
# ruby_test.rb:52): as there, inserts and include? raise ArgumentError; an unknown
# engine raises NoMethodError, as `send("engine_#{engine}")` does.
require_relative 'hip'

class Redis
  module BloomfilterDriver
    class HipTest < Hip
      ENGINES = { 'md5' => HipFFI::BF_FLAG_ENGINE_MD5, 'sha1' => HipFFI::BF_FLAG_ENGINE_SHA1 }.freeze

      def insert_many(keys, expire = nil)
        check_engine
        super
      end

      def include_many?(keys)
        check_engine
        super
      end

      protected

      def config_flags
        @engine = (@options[:hash_engine] || 'md5').to_s
        ENGINES.fetch(@engine, HipFFI::BF_FLAG_ENGINE_MD5)
      end

      private

      def check_engine
        return if ENGINES.key?(@engine)
        raise ArgumentError, 'wrong number of arguments (given 1, expected 0)' if @engine == 'crc32'

        raise NoMethodError, "undefined method `engine_#{@engine}' for #{self.class}"
      end
    end
  end
end
